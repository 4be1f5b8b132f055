// Minimal HIP program (no torch, no librvhip): does ROCm's stream capture
// survive the fork pattern the round-2 pipelined step graphs used?
//
// In those graphs the YOLO forward's second half ran on a capturing stream
// and forked the Detect heads onto the model's own side streams
// (hipEventRecord on the capturing stream, hipStreamWaitEvent on a side
// stream created with hipStreamNonBlocking, kernels there, an event back),
// and the whole stage was itself a branch forked from the capture origin;
// the same fork / join event objects were re-recorded once per pipeline
// stage.  Round 2 saw host-side SIGSEGVs in hipStreamEndCapture and
// hipGraphLaunch of those graphs.
//
// mode 0: one-level fork  origin -> B            (control)
// mode 1: nested fork     origin -> B -> C1, C2  (fresh events per stage)
// mode 2: nested fork, the SAME fork / join events re-recorded every stage
//         (what the forward's head fork did: one event pair per side stream)
// Each mode captures `stages` stages into one graph, instantiates it and
// replays it `reps` times; prints one line per phase so a crash names it.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      fflush(stdout);                                                          \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void axpy(float* y, const float* x, int n, float a) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * y[i] + x[i];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int stages = argc > 2 ? atoi(argv[2]) : 8;
  const int reps = argc > 3 ? atoi(argv[3]) : 200;
  const int n = 1 << 18;
  float *x, *y[4];
  CK(hipMalloc(&x, n * 4));
  for (int i = 0; i < 4; ++i) CK(hipMalloc(&y[i], n * 4));
  CK(hipMemset(x, 0, n * 4));
  hipStream_t origin, B, C[2];
  CK(hipStreamCreate(&origin));
  CK(hipStreamCreate(&B));
  for (int i = 0; i < 2; ++i) CK(hipStreamCreateWithFlags(&C[i], hipStreamNonBlocking));
  hipEvent_t fixed_fork[2], fixed_join[2];
  for (int i = 0; i < 2; ++i) {
    CK(hipEventCreateWithFlags(&fixed_fork[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&fixed_join[i], hipEventDisableTiming));
  }
  std::vector<hipEvent_t> evs;
  auto ev = [&]() {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return (hipEvent_t) nullptr;
    evs.push_back(e);
    return e;
  };
  const dim3 g((n + 255) / 256), b(256);
  printf("mode %d: capture of %d stages\n", mode, stages);
  fflush(stdout);
  CK(hipStreamBeginCapture(origin, hipStreamCaptureModeGlobal));
  for (int s = 0; s < stages; ++s) {
    hipEvent_t f = ev(), j = ev();
    CK(hipEventRecord(f, origin));
    CK(hipStreamWaitEvent(B, f, 0));
    axpy<<<g, b, 0, origin>>>(y[0], x, n, 0.5f);
    axpy<<<g, b, 0, B>>>(y[1], x, n, 0.5f);
    if (mode >= 1) {  // B forks two side streams, as the forward forked its heads
      for (int i = 0; i < 2; ++i) {
        hipEvent_t ff = mode == 2 ? fixed_fork[i] : ev();
        hipEvent_t jj = mode == 2 ? fixed_join[i] : ev();
        CK(hipEventRecord(ff, B));
        CK(hipStreamWaitEvent(C[i], ff, 0));
        axpy<<<g, b, 0, C[i]>>>(y[2 + i], x, n, 0.25f);
        CK(hipEventRecord(jj, C[i]));
        axpy<<<g, b, 0, B>>>(y[1], x, n, 0.5f);
        CK(hipStreamWaitEvent(B, jj, 0));
      }
    }
    axpy<<<g, b, 0, B>>>(y[1], x, n, 0.5f);
    CK(hipEventRecord(j, B));
    CK(hipStreamWaitEvent(origin, j, 0));
  }
  hipGraph_t graph;
  CK(hipStreamEndCapture(origin, &graph));
  printf("end capture ok\n");
  fflush(stdout);
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  printf("instantiate ok\n");
  fflush(stdout);
  for (int r = 0; r < reps; ++r) {
    CK(hipGraphLaunch(exec, origin));
    if (r % 50 == 0) {
      CK(hipStreamSynchronize(origin));
      printf("replay %d ok\n", r);
      fflush(stdout);
    }
  }
  CK(hipStreamSynchronize(origin));
  printf("mode %d: %d replays ok\n", mode, reps);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return 0;
}
