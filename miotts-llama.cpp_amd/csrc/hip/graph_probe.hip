// Diagnostic: a graph of `nodes` empty launches (one 64-thread workgroup each) replayed
// `replays` times on the device's stream. It separates the graph-replay machinery from the
// decode step's kernels: run under `rocprofv3 --kernel-trace`, it shows whether the profiler's
// fault after ~28k intercepted replays needs anything of ours; timed alone, it
// gives the per-node floor of a replayed graph on this box.
#include <hip/hip_runtime.h>

#include <chrono>

#include "common.h"

namespace {
__global__ __launch_bounds__(64) void k_nop(int *sink, int v) {
    if (sink && v < 0) sink[threadIdx.x] = v;  // never taken: the launch does nothing
}
}  // namespace

extern "C" int mio_hip_debug_graph_replay(mio_hip_device *d, int replays, int nodes, double *wall_ms) {
    MIO_REQUIRE(d && wall_ms && replays > 0 && nodes > 0 && nodes <= 4096, MIO_ERR_INVALID,
                "debug_graph_replay: bad args");
    int rc = mio::bind(d);
    if (rc) return rc;
    hipStream_t s = d->stream;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    MIO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < nodes; ++i) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, (int *)nullptr, i);
    MIO_HIP_CHECK(hipStreamEndCapture(s, &g));
    MIO_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    MIO_HIP_CHECK(hipGraphLaunch(ge, s));  // warm
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipSuccess;
    for (int r = 0; r < replays && e == hipSuccess; ++r) e = hipGraphLaunch(ge, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    *wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    hipGraphExecDestroy(ge);
    MIO_HIP_CHECK(e);
    return MIO_OK;
}
