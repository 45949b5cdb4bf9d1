// Cost of a dependent kernel boundary inside a captured HIP graph on one stream: N
// kernels that read a device flag and return (the shape of a converged superstep's
// empty launches), for several grid sizes, against the same N launches eagerly; and
// the same chain split over two forked streams.  Prints one line per case: us per
// kernel (graph replay time / N).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb_launch tools/microbench/mb_launch.hip && /tmp/mb_launch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void k_flag(const int* __restrict__ flag, int* __restrict__ out) {
  if (*flag) out[blockIdx.x] = threadIdx.x;  // never taken (flag is 0)
}

static float time_graph(hipGraphExec_t ge, hipStream_t s, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main() {
  int *flag, *out;
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(flag, 0, 4));
  CK(hipMalloc(&out, 1 << 20));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  const int grids[] = {1, 64, 256, 1024, 2048, 8192};
  const int N = 24, reps = 200;
  for (int gi = 0; gi < 6; ++gi) {
    const int gr = grids[gi];
    // one stream, N dependent launches
    hipGraph_t gph;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_flag, dim3(gr), dim3(256), 0, s, flag, out);
    CK(hipStreamEndCapture(s, &gph));
    CK(hipGraphInstantiate(&ge, gph, nullptr, nullptr, 0));
    const float one = time_graph(ge, s, reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gph));
    // the same N launches split N/2 + N/2 over two forked streams
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, s));
    CK(hipStreamWaitEvent(s2, fork, 0));
    for (int k = 0; k < N / 2; ++k) {
      hipLaunchKernelGGL(k_flag, dim3(gr), dim3(256), 0, s, flag, out);
      hipLaunchKernelGGL(k_flag, dim3(gr), dim3(256), 0, s2, flag, out);
    }
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s, join, 0));
    CK(hipStreamEndCapture(s, &gph));
    CK(hipGraphInstantiate(&ge, gph, nullptr, nullptr, 0));
    const float two = time_graph(ge, s, reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gph));
    // eager launches
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 20; ++r)
      for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_flag, dim3(gr), dim3(256), 0, s, flag, out);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("grid %5d: graph 1 stream %.2f us/kernel, graph 2 streams %.2f us/kernel-pair-slot, eager %.2f us/kernel\n",
           gr, 1e3f * one / N, 1e3f * two / (N / 2), 1e3f * ms / (20 * N));
    fflush(stdout);
  }
  CK(hipFree(flag));
  CK(hipFree(out));
  return 0;
}
