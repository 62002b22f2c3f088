// Parameter-server gradient-collection state machine (SURVEY.md §2.6 PAR-DP-PS / KILL / BACKUP).
//
// Transport-agnostic: the master feeds it "worker w delivered layer l for step s" events (from RCCL
// completions, store keys or the native MLP's messages) and asks when the step may close.
//
// Modes, matching the reference's intended behaviour (not its bugs):
//  * full sync (PT-02n, PP-02n): close when every layer has all n_workers contributions.
//  * k-of-n kill (PT-02): once `kill_k` workers delivered the SENTINEL layer (the reference counts
//    parameter 0 = the last gradient a worker sends, sync_replicas_master_nn.py:172-186) the step closes
//    and every worker that has not delivered it is a straggler to be killed.  Averages must use the real
//    per-layer count (pdnn_ps_count), fixing defect D3 (divide by N-1 regardless).
//  * backup workers (CPP-03): close when every layer has >= n_to_collect fresh gradients; gradients
//    tagged with an older step are dropped as stale (sync_replicas_master_nn.h:85).
//  Duplicate deliveries (same worker/layer/step) are ignored, fixing the ANY_SOURCE slot race D2.
//  Every accepted arrival is time-stamped for the arrival timeline (CPP-03 GENERATE_TIMELINE,
//  MPI_code/src/python/visualize_timeline.py).
#include "runtime.h"

#include <vector>

namespace {
struct Arrival {
    double t;
    int64_t step;
    int worker, layer;
};

struct PS {
    int n_workers, n_layers, n_to_collect, kill_k;
    int64_t step = 0;
    int64_t stale = 0;
    bool closed = false;
    std::vector<std::vector<uint8_t>> got;   // [layer][worker]
    std::vector<int> count;
    std::vector<Arrival> timeline;

    PS(int nw, int nl, int nc, int k) : n_workers(nw), n_layers(nl), n_to_collect(nc), kill_k(k) { begin(0); }

    void begin(int64_t s) {
        step = s;
        closed = false;
        got.assign(n_layers, std::vector<uint8_t>(n_workers, 0));
        count.assign(n_layers, 0);
    }

    // 0 accepted, 1 stale (older step), 2 duplicate, 3 step already closed, 4 bad index, 5 future step
    int offer(int w, int l, int64_t s, double t) {
        if (w < 0 || w >= n_workers || l < 0 || l >= n_layers) return 4;
        if (s < step) { ++stale; return 1; }
        if (s > step) return 5;
        if (closed) return 3;
        if (got[l][w]) return 2;
        got[l][w] = 1;
        ++count[l];
        timeline.push_back({t, s, w, l});
        return 0;
    }

    bool done() {
        if (closed) return true;
        bool ok = true;
        if (kill_k > 0) {
            // sentinel = layer 0 (the last gradient a worker produces in backward order)
            ok = count[0] >= kill_k;
        } else {
            const int need = n_to_collect > 0 ? n_to_collect : n_workers;
            for (int l = 0; l < n_layers; ++l) ok = ok && count[l] >= need;
        }
        if (ok) closed = true;
        return ok;
    }
};
}  // namespace

extern "C" {
RT_API void* pdnn_ps_create(int n_workers, int n_layers, int n_to_collect, int kill_k) {
    if (n_workers <= 0 || n_layers <= 0) return nullptr;
    return new PS(n_workers, n_layers, n_to_collect, kill_k);
}
RT_API void pdnn_ps_destroy(void* h) { delete static_cast<PS*>(h); }
RT_API void pdnn_ps_begin_step(void* h, int64_t step) { static_cast<PS*>(h)->begin(step); }
RT_API int pdnn_ps_offer(void* h, int worker, int layer, int64_t step, double t_ms) {
    return static_cast<PS*>(h)->offer(worker, layer, step, t_ms);
}
RT_API int pdnn_ps_done(void* h) { return static_cast<PS*>(h)->done() ? 1 : 0; }
// close the step from outside the count rule (interval / deadline): later offers return 3 (closed)
RT_API void pdnn_ps_close(void* h) { static_cast<PS*>(h)->closed = true; }
RT_API int pdnn_ps_count(void* h, int layer) {
    auto* p = static_cast<PS*>(h);
    return (layer >= 0 && layer < p->n_layers) ? p->count[layer] : -1;
}
RT_API int pdnn_ps_stragglers(void* h, int sentinel_layer, int* out) {
    auto* p = static_cast<PS*>(h);
    int n = 0;
    for (int w = 0; w < p->n_workers; ++w)
        if (!p->got[sentinel_layer][w]) out[n++] = w;
    return n;
}
RT_API int pdnn_ps_contributed(void* h, int layer, int worker) {
    return static_cast<PS*>(h)->got[layer][worker];
}
RT_API int64_t pdnn_ps_stale_dropped(void* h) { return static_cast<PS*>(h)->stale; }
RT_API int pdnn_ps_timeline(void* h, double* t, int64_t* step, int* worker, int* layer, int cap) {
    auto* p = static_cast<PS*>(h);
    int n = 0;
    for (const auto& a : p->timeline) {
        if (n >= cap) break;
        t[n] = a.t;
        step[n] = a.step;
        worker[n] = a.worker;
        layer[n] = a.layer;
        ++n;
    }
    return (int)p->timeline.size();
}
}
