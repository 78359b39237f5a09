// Diagnostic tool (not part of libmiotts.so): a graph of `nodes` empty launches (one
// 64-thread workgroup each) replayed `replays` times. It separates the graph-replay machinery
// from the decode step's kernels: run under `rocprofv3 --kernel-trace`, it shows whether the
// profiler's fault after ~28k intercepted replays needs anything of ours; timed
// alone, it gives the per-node floor of a replayed graph on this box.
//   make -C tools/micro graph_probe && tools/micro/graph_probe [replays] [nodes]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s -> %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ __launch_bounds__(64) void k_nop(int *sink, int v) {
    if (sink && v < 0) sink[threadIdx.x] = v;  // never taken: the launch does nothing
}

int main(int argc, char **argv) {
    const int replays = argc > 1 ? std::atoi(argv[1]) : 1000;
    const int nodes = argc > 2 ? std::atoi(argv[2]) : 1;
    if (replays <= 0 || nodes <= 0 || nodes > 4096) return 2;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < nodes; ++i) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, (int *)nullptr, i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    CK(hipGraphLaunch(ge, s));  // warm
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < replays; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"replays\": %d, \"nodes\": %d, \"wall_ms\": %.3f, \"us_per_node\": %.3f}\n", replays, nodes, ms,
                1000.0 * ms / ((double)replays * nodes));
    CK(hipGraphExecDestroy(ge));
    CK(hipStreamDestroy(s));
    return 0;
}
