"""CPU oracle for the STIF hot path -- TEST INFRASTRUCTURE ONLY (see stif_oracle.py)."""
