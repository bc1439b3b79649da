"""Reference-compatible facade (`utils.*`)."""
