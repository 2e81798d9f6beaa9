// Stand-alone check of HIP stream capture across N streams (round 6 diagnosis of the
// multi-stream multi-model capture, fortran_abi.hip): stream 0 begins a capture, the others
// join by events, each stream launches kernels and device-to-device copies, B all-to-all event
// barriers cross the streams, every stream joins back, then hipStreamEndCapture, instantiate,
// launch, synchronise.  Prints each stage; pass N and B on the command line.
//   hipcc --offload-arch=gfx950 -O2 tools/capture_repro.hip -o tools/capture_repro
//   tools/capture_repro N B [kc|k|c] [global|relaxed]
// The third argument keeps the kernels (k), the copies (c) or both (kc, default); the fourth
// picks the capture mode.  With f in the third argument the B barriers are replaced by one
// fan-in: every stream launches, stream 0 waits for the others' events and launches one kernel,
// whose graph node then has N dependencies.  With e instead: stream 0 waits for the others'
// events, records an event with no node of its own after the waits (the event then stands for
// all N streams' last nodes), and stream 1 waits for it and launches.  With n (barrier form) a
// one-thread kernel follows every stream's barrier waits, so no event is ever recorded on a
// stream whose last captured operation is a wait.  With o: stream 0 launches, records an
// event, the other streams wait for it and launch, stream 0 launches again (one node with N
// dependents).  With g the B barriers go through stream 0: it waits for the others' events,
// launches a one-thread kernel and records an event the others wait for.
#include <cstring>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void k_nop(double *y) {
  if (threadIdx.x == 1000) y[0] = 0.0;
}

__global__ void k_axpy(double *y, const double *x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] + 0.5 * x[i];
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 4, B = argc > 2 ? atoi(argv[2]) : 4, n = 1 << 16;
  const char *what = argc > 3 ? argv[3] : "kc";
  const bool kern = strchr(what, 'k') != nullptr, copy = strchr(what, 'c') != nullptr;
  const bool fan = strchr(what, 'f') != nullptr, evset = strchr(what, 'e') != nullptr;
  const bool nop = strchr(what, 'n') != nullptr, fout = strchr(what, 'o') != nullptr;
  const bool gather = strchr(what, 'g') != nullptr;
  const bool relaxed = argc > 4 && strcmp(argv[4], "relaxed") == 0;
  std::vector<hipStream_t> s(N);
  std::vector<double *> a(N), b(N);
  for (int i = 0; i < N; i++) {
    CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    CK(hipMalloc(&a[i], n * sizeof(double)));
    CK(hipMalloc(&b[i], n * sizeof(double)));
    CK(hipMemset(a[i], 0, n * sizeof(double)));
    CK(hipMemset(b[i], 0, n * sizeof(double)));
  }
  std::vector<hipEvent_t> ev;   // one event per record (none recorded twice)
  auto newev = [&]() {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) abort();
    ev.push_back(e);
    return e;
  };
  CK(hipDeviceSynchronize());
  printf("N=%d B=%d %s %s: begin capture\n", N, B, what, relaxed ? "relaxed" : "global");
  fflush(stdout);
  CK(hipStreamBeginCapture(s[0], relaxed ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal));
  hipEvent_t f = newev();
  CK(hipEventRecord(f, s[0]));
  for (int i = 1; i < N; i++) CK(hipStreamWaitEvent(s[i], f, 0));
  if (fan) {
    std::vector<hipEvent_t> e(N);
    for (int i = 0; i < N; i++) {
      hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[i], a[i], b[i], n);
      e[i] = newev();
      CK(hipEventRecord(e[i], s[i]));
    }
    for (int j = 1; j < N; j++) CK(hipStreamWaitEvent(s[0], e[j], 0));
    hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[0], a[0], b[0], n);
  }
  if (evset) {
    std::vector<hipEvent_t> e(N);
    for (int i = 0; i < N; i++) {
      hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[i], a[i], b[i], n);
      e[i] = newev();
      CK(hipEventRecord(e[i], s[i]));
    }
    for (int j = 1; j < N; j++) CK(hipStreamWaitEvent(s[0], e[j], 0));
    hipEvent_t g = newev();
    CK(hipEventRecord(g, s[0]));
    CK(hipStreamWaitEvent(s[1], g, 0));
    hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[1], a[1], b[1], n);
  }
  if (fout) {
    hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[0], a[0], b[0], n);
    hipEvent_t g = newev();
    CK(hipEventRecord(g, s[0]));
    for (int i = 1; i < N; i++) {
      CK(hipStreamWaitEvent(s[i], g, 0));
      hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[i], a[i], b[i], n);
    }
    hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[0], a[0], b[0], n);
  }
  for (int r = 0; r < (fan || evset || fout ? 0 : B); r++) {
    for (int i = 0; i < N; i++) {
      if (kern) hipLaunchKernelGGL(k_axpy, dim3(n / 256), dim3(256), 0, s[i], a[i], b[i], n);
      if (copy) CK(hipMemcpyAsync(b[(i + 1) % N], a[i], n * sizeof(double), hipMemcpyDeviceToDevice, s[i]));
    }
    std::vector<hipEvent_t> e(N);
    for (int i = 0; i < N; i++) {
      e[i] = newev();
      CK(hipEventRecord(e[i], s[i]));
    }
    if (gather) {
      for (int j = 1; j < N; j++) CK(hipStreamWaitEvent(s[0], e[j], 0));
      hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s[0], a[0]);
      hipEvent_t g = newev();
      CK(hipEventRecord(g, s[0]));
      for (int i = 1; i < N; i++) CK(hipStreamWaitEvent(s[i], g, 0));
    } else {
      for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++)
          if (i != j) CK(hipStreamWaitEvent(s[i], e[j], 0));
    }
    if (nop)
      for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s[i], a[i]);
  }
  for (int i = 1; i < N; i++) {
    hipEvent_t e = newev();
    CK(hipEventRecord(e, s[i]));
    CK(hipStreamWaitEvent(s[0], e, 0));
  }
  printf("N=%d B=%d: joined, ending capture\n", N, B);
  fflush(stdout);
  hipGraph_t g;
  CK(hipStreamEndCapture(s[0], &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  printf("N=%d B=%d: captured %zu nodes\n", N, B, nn);
  fflush(stdout);
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, s[0]));
  CK(hipStreamSynchronize(s[0]));
  printf("N=%d B=%d: replayed ok\n", N, B);
  return 0;
}
