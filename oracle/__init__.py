"""CPU oracle package -- test infrastructure only (see sketch_oracle.h)."""
