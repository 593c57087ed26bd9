"""Stub package (see ../README.md)."""
