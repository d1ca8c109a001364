"""CPU oracle (test infrastructure only). See tpe_oracle.py."""
