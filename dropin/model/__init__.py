"""Overlay package ``model`` (see dropin/sitecustomize.py)."""
