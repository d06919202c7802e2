"""CPU oracle for ddr_amd parity tests.  TEST INFRASTRUCTURE ONLY -- never imported by ddr_amd."""
