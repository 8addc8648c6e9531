// ring_kernels.hip -- the resident per-call ring's kernel (ring_kernel,
// launch_ring; host side ring.cpp).  gso_kernels.hip's device code compiled
// once more with WGCS_RING_TU: every load of request bytes is a system-scope
// one (wgcs_copy.h: ld16 / ldg8 relaxed atomics, buffer loads sc0 sc1), since
// the kernel stays resident while the host rewrites the same buffers between
// requests and a plain load may hit the CU's L1 copy of the last request.
// The batch kernels are compiled in gso_kernels.hip's own translation unit.
#define WGCS_RING_TU 1
#include "gso_kernels.hip"
