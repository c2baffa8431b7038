"""ORACLE package — test infrastructure only (see oracle/kma_oracle.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
