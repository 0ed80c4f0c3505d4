"""ORACLE — test infrastructure only (see clip_ref.py header). Not part of the product path."""
