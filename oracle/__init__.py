"""TEST INFRASTRUCTURE ONLY: CPU oracle of the reference frame (see drone_oracle.c)."""
