"""ORACLE package — test infrastructure only (see reference_ops.py header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product (verl_amd/) never imports it.
"""
