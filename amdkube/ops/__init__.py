"""Native / GPU operations used by the control plane and the validation workloads.

  topology  — xGMI/NUMA GPU-subset selection (C++ `_topo`, Python reference)
  hip       — in-process HIP (gfx950) kernels: vector add, HBM probe, MFMA burn (`_hipops`)
"""
