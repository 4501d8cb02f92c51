"""CPU restatement of the reference rasterizer -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  See oracle/gsr_oracle.c for the restatement and its citations.
"""
