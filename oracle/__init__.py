"""CPU oracle -- TEST INFRASTRUCTURE ONLY (see tis_oracle.c header)."""
