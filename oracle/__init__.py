"""CPU oracle — TEST INFRASTRUCTURE ONLY (see oracle/als_oracle.py).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker.  The product never imports it.
"""
