"""TEST INFRASTRUCTURE ONLY — CPU oracle for the RS hot path (see README.md).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, as the checker; the product never does.
"""
