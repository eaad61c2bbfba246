// dual_regs.hip -- one exact local-optimum kernel alone (nemo_exact.hip), for
// its register / scratch report and ISA without the library's other kernels:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I nem-mcmc-optimization_amd/csrc -c \
//         tools/ubench/dual_regs.hip -Rpass-analysis=kernel-resource-usage [-save-temps]
// (-DWHICH=0: the dual form, NS = 2; 1: the cached throughput form; 2 throughput; 3 latency)
#define NEMO_EXACT_KERNELS_ONLY
#include "nemo_exact.hip"
#ifndef WHICH
#define WHICH 0
#endif
namespace nemo {
#if WHICH == 0
const void* probe_kernel = (const void*)&local_opt_exact_dual_kernel<2>;
#elif WHICH == 1
const void* probe_kernel = (const void*)&local_opt_exact_kernel<2, false, true, true>;
#elif WHICH == 2
const void* probe_kernel = (const void*)&local_opt_exact_kernel<2, false, true>;   // throughput
#else
const void* probe_kernel = (const void*)&local_opt_exact_kernel<2, true, true>;    // latency + cache
#endif
}
