"""RPN custom ops facade."""
