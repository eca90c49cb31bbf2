"""aby3_amd: MI355X-native local-compute engine for ABY3's replicated
secret-sharing hot path.

* ``include/aby3gpu.h`` / ``aby3_amd/lib/libaby3gpu.so`` -- HIP kernels (gfx950)
  behind a C-ABI.
* ``include/aby3.h`` / ``aby3_amd/lib/libaby3.so`` -- the C++ host runtime that
  mirrors the reference's Sh3Runtime / Sh3Encryptor / Sh3Evaluator /
  Sh3BinaryEvaluator / Sh3Piecewise API.
* ``aby3_amd.native`` -- ctypes binding of the C-ABI (tests, bench).
"""
