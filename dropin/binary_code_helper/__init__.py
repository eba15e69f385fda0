"""Overlay package ``binary_code_helper`` (see dropin/sitecustomize.py)."""
