"""CPU oracle for the StableKeypoints hot path — test infrastructure only (see skp_oracle.py)."""
