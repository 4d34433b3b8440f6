"""CPU oracle for the self-play hot path. TEST INFRASTRUCTURE ONLY (see spec.py)."""
