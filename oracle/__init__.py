"""Oracle package — TEST INFRASTRUCTURE ONLY (see rt_oracle.c header).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Parity status: unpinned by the reference (Go toolchain absent; no reference fixtures).
"""
