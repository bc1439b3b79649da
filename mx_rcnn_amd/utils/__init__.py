"""Persistence (MXNet .params codec, checkpoints, combine) and profiling utilities."""
