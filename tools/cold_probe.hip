// Cold-start probe (tools only): a one-kernel library, to separate the first-launch cost of a
// code object of one kernel from that of libcc_mi355x.so's (tools/cold_probe.py).
#include <hip/hip_runtime.h>
__global__ void k_probe(int* p) { if (threadIdx.x == 0) p[0] += 1; }
extern "C" int probe_launch(void* stream, int* p) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
    return (int)hipGetLastError();
}
