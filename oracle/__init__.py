"""CPU oracle of the transfer step — test infrastructure only (see pmmg_oracle.h)."""
