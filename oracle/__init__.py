"""CPU oracle for the Eden codec path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker.  The product path (openfl_amd/) never
imports it.  See eden_oracle.c for the function-by-function citation of
/root/reference/openfl/pipelines/eden_pipeline.py that it restates, and
tests/test_oracle_golden.py for how it is pinned to the reference's outputs.
"""
