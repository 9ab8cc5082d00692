"""Bench/test tooling (synthetic frame generation on the GPU)."""
