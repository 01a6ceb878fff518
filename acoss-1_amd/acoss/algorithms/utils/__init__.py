"""Pairwise helpers (acoss/algorithms/utils), backed by the HIP engine."""
