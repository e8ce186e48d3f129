"""CPU oracle -- TEST INFRASTRUCTURE ONLY (see gcn_oracle.py header)."""
