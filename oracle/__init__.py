"""TEST INFRASTRUCTURE ONLY — see oracle/hdx_oracle.h.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (hyperdex_amd/) never does.
"""
