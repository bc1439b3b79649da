"""Host-side (numpy) geometry primitives with the reference's exact semantics.

These mirror `helper/processing/*.py` of the reference and are used by the
roidb / dataset pipeline and as test oracles.  The device hot path uses the
HIP kernels in :mod:`mx_rcnn_amd.ops` instead.
"""
