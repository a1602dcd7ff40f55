"""CPU oracle for the ZNCC stereo cost volume -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this package, and only as the checker / the timed
CPU baseline.  The product package ``custereomatching_amd`` never imports it
(tests/test_no_oracle_in_product.py enforces that).

Contents
  * ``zncc_oracle.c`` / ``liborc.so`` -- C restatement of the reference CUDA
    arithmetic (custma/src/stereo_matching_kernel.cu:4-179).
  * ``oracle.py`` -- numpy/ctypes wrappers around it.
  * ``torch_ref.py`` -- restatement of the reference's PyTorch CPU path
    (examples/verify.py:18-28, 81-133): unfold + bmm + autograd.

Parity pinning: the C restatement is checked against golden vectors made by
importing the reference's own ``examples/verify.py`` (tests/golden/gen_golden.py).
The reference CUDA extension itself is unbuildable here (needs nvcc and
CUDA headers), so no ``oracle/_ref`` binary exists; see DESIGN.md.
"""
