"""Reference-compatible facade (`helper.*`)."""
