"""TEST INFRASTRUCTURE ONLY: CPU oracle for the rx transform (see oracle.py)."""
