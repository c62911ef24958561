"""CPU oracle for the hot path -- TEST INFRASTRUCTURE ONLY (see oracle.py / mzh_oracle.c)."""
