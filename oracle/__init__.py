"""CPU oracle for the sclmd GLE hot path -- TEST INFRASTRUCTURE ONLY (see sclmd_oracle.py)."""
