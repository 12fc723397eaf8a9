"""Shared serving of one model to the co-located clients of a GPU share group."""
from .client import generate  # noqa: F401
