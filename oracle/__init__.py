"""CPU oracle for the Reed-Solomon path -- TEST INFRASTRUCTURE ONLY.

Restates the reference codec (Backblaze JavaReedSolomon as vendored in
/root/reference/src/main/java/edu/cmu/reedsolomon/) twice: in C (rs_oracle.c,
loaded by c_ref.py) and in numpy (numpy_ref.py).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only
as the checker.  The product package never imports it.
"""
