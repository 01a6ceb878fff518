"""Cover-ID algorithms (acoss/algorithms), backed by the HIP engine."""
