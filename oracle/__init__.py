"""CPU oracle for the digital-filter + PODFS hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import anything from here, and only as the checker / the timed
CPU baseline -- never as the product path.  See oracle/pods_oracle.py.
"""
