// Cross-stream ordering for the two-stream ResNet schedule (ops/fused_resnet.py: weight gradients on a side
// stream, the data-gradient chain on the compute stream, ~70 fork / join points per step).
//
// torch's Stream.wait_stream records a default HIP event (system-scope release when it is reached: a
// write-back + invalidate of the caches) and makes the other stream wait on it.  Every such marker left a
// ~7 us bubble on the compute stream (profiles/resnet50_bs256_timeline_r3c.txt: 71 idle gaps, 627 us per
// step, against ~1-2 us between plain back-to-back kernels).  Both streams here live on one device, and
// each kernel's own end-of-dispatch release already makes its results visible device-wide, so the marker
// needs no system-scope fence: these events are created with hipEventDisableSystemFence (and no timing).
// Measured (dev/gpu_runs/archive_r1_r3.txt "r3_58", same box): median compute-stream gap 7.3 -> 5.5 us, ResNet-50
// 10,604-10,615 -> 10,687-10,689 img/s.
#include "common.h"

#include <mutex>

namespace {
constexpr int EV_RING = 256;          // events per device; a wait captures the record it follows, so a
constexpr int EV_DEVS = 16;           // slot can be re-recorded once later waits have been enqueued
hipEvent_t g_ring[EV_DEVS][EV_RING];
unsigned g_next[EV_DEVS];
bool g_init[EV_DEVS];
std::mutex g_mu;                      // the autograd engine's device threads and the forward thread
}  // namespace

// `waiter` runs its later work only after everything enqueued on `signaler` so far (same device).
PDNN_API int pdnn_stream_wait(hipStream_t waiter, hipStream_t signaler) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= EV_DEVS) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_init[dev]) {
        for (int i = 0; i < EV_RING; ++i) {
            e = hipEventCreateWithFlags(&g_ring[dev][i], hipEventDisableTiming | hipEventDisableSystemFence);
            if (e != hipSuccess) return (int)e;
        }
        g_init[dev] = true;
    }
    hipEvent_t ev = g_ring[dev][g_next[dev]++ % EV_RING];
    e = hipEventRecord(ev, signaler);
    if (e != hipSuccess) return (int)e;
    return (int)hipStreamWaitEvent(waiter, ev, 0);
}

// Experimental alternative fork (tools/fork_cost.py only): a stream-ordered 32-bit write on `signaler` and a
// wait-until->= on `waiter` over one word of signal memory per device.  Values increase monotonically per
// device.  Cheaper than an event in the tiny-kernel microbenchmark (11.7 vs 12.4 us per link), but the
// ResNet-50 step ran 6-7% slower with it (gpurun_out/r3_61): not used by the framework.
namespace {
unsigned* g_sig[EV_DEVS];
unsigned g_sig_next[EV_DEVS];
}  // namespace

PDNN_API int pdnn_stream_wait_value(hipStream_t waiter, hipStream_t signaler) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= EV_DEVS) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_sig[dev]) {
        void* p = nullptr;
        e = hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory);   // signal memory: exactly 8 bytes
        if (e != hipSuccess) return (int)e;
        g_sig[dev] = static_cast<unsigned*>(p);
        e = hipMemset(p, 0, 8);
        if (e != hipSuccess) return (int)e;
        e = hipDeviceSynchronize();
        if (e != hipSuccess) return (int)e;
    }
    const unsigned v = ++g_sig_next[dev];
    e = hipStreamWriteValue32(signaler, g_sig[dev], v, 0);
    if (e != hipSuccess) return (int)e;
    return (int)hipStreamWaitValue32(waiter, g_sig[dev], v, hipStreamWaitValueGte, 0xffffffffu);
}
