"""CPU oracle for the hhfm_amd hot path — TEST INFRASTRUCTURE ONLY.

Restatement of the reference's scoring graphs (numpy: fm_oracle.py; C +
OpenMP: cpu_oracle.c via cpu.py).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker —
never by the product package hhfm_amd.
"""
