// Native MLP trainer + parameter-server roles (reference
// MPI_code/src/nn/{nn,nn_layer,nn_params}.h, MPI_code/src/util/util.h,
// MPI_code/src/distributed/{sync_replicas_master_nn,worker_nn,evaluator_nn}.h).
//
// Model: dense layers with the bias folded in as the last weight row ((n_in+1) x n_out) and a ones
// column appended to every activation (nn_layer.h:46-50); sigmoid hidden units whose derivative is
// produced in the same pass (nn_layer.h:130-134); softmax output with the fused (p - onehot)/B
// gradient (nn_layer.h:150-152); plain SGD W -= lr*G (nn_layer.h:78-83).  GEMMs are a cache-blocked
// kernel templated on the precision: fp32 by default, fp64 with --fp64 / the *_ex(fp64=1) entry points, which
// is the reference's own arithmetic (cblas_dgemm over doubles, util.h:35-81).
//
// Distributed roles over the control-plane store (the reference uses MPI p2p with per-layer
// communicators; here every message is a store key):
//   step                      int64, current global step (-1 = shut down)          [C-08 / C-11]
//   w/<step>/<layer>          weights of a layer for that step                     [C-09]
//   g/<step>/<layer>/<worker> a worker's gradient of a layer for that step         [C-10]
//   gq_n, gq/<n>              arrival queue: "<step> <layer> <worker>" per pushed gradient
//   go/<step>                 opened steps (blocking waits of workers / evaluator)  [C-08]
//   scheme                    run name for the evaluator's output file             [C-12]
// Master: publishes step + weights, then BLOCKS on the arrival queue (the store-side MPI_Waitany of
// sync_replicas_master_nn.h:66-74; no polling) and feeds every announced gradient to the PS coordinator
// (backup workers: n_to_collect); a gradient of an older step -- a late worker of a closed step -- is
// dropped by its step tag (:85) and its key deleted, so nothing leaks; applies ApplyGrad(lr / count)
// (:124-128).
// Worker: layer-pipelined forward (fetch layer i's weights just before computing it, worker_nn.h:66-70),
// pushes each layer's gradient as soon as it exists, and SHORT-CIRCUITS (abandons the iteration)
// whenever a newer step is published (worker_nn.h:59-64, 79-84).
// Evaluator: on every new step evaluates the full test set and appends "step time_ms loss err" to
// <out_prefix>time_loss_out_<scheme> (evaluator_nn.h:55-58).
#include "runtime.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

// C[M][N] (+)= A[M][K] * B[K][N], all row-major; optional transposes via strides.  Blocked over (k, n);
// a transposed B block is packed k-major first so the inner loop is a contiguous axpy the compiler
// vectorises (the strided B[j][k] walk was the slow path of the data-gradient GEMM).
template <typename T>
void gemm(int M, int N, int K, const T* A, int lda, bool ta, const T* B, int ldb, bool tb, T* C,
          int ldc, bool accumulate) {
    if (!accumulate)
        for (int i = 0; i < M; ++i) std::fill(C + (long)i * ldc, C + (long)i * ldc + N, T(0));
    constexpr int BK = 64, BN = 256;
    std::vector<T> pack(tb ? (size_t)BK * BN : 0);
    for (int k0 = 0; k0 < K; k0 += BK) {
        const int k1 = std::min(K, k0 + BK);
        for (int n0 = 0; n0 < N; n0 += BN) {
            const int n1 = std::min(N, n0 + BN), nw = n1 - n0;
            const T* bblk;
            long bld;
            if (tb) {
                for (int j = n0; j < n1; ++j)
                    for (int k = k0; k < k1; ++k) pack[(size_t)(k - k0) * nw + (j - n0)] = B[(long)j * ldb + k];
                bblk = pack.data() - (long)k0 * nw - n0;
                bld = nw;
            } else {
                bblk = B;
                bld = ldb;
            }
            for (int i = 0; i < M; ++i) {
                T* c = C + (long)i * ldc;
                for (int k = k0; k < k1; ++k) {
                    const T a = ta ? A[(long)k * lda + i] : A[(long)i * lda + k];
                    if (a == T(0)) continue;
                    const T* b = bblk + (long)k * bld;
                    for (int j = n0; j < n1; ++j) c[j] += a * b[j];
                }
            }
        }
    }
}

template <typename T>
struct LayerT {
    int nin, nout;
    std::vector<T> W, G;   // (nin+1) x nout
};

template <typename T>
struct MLPT {
    std::vector<int> sizes;
    int batch;
    float lr;
    std::vector<LayerT<T>> layers;
    std::vector<std::vector<T>> Z, F, D;   // activations (with ones column), derivatives, deltas

    MLPT(const int* s, int n, int b, float lr_, uint64_t seed) : sizes(s, s + n), batch(b), lr(lr_) {
        std::mt19937_64 rng(seed);
        std::normal_distribution<float> nd(0.f, 1.f);
        for (int i = 0; i + 1 < n; ++i) {
            LayerT<T> L;
            L.nin = s[i];
            L.nout = s[i + 1];
            L.W.resize((size_t)(L.nin + 1) * L.nout);
            L.G.assign(L.W.size(), T(0));
            const float std_ = 1.f / std::sqrt((float)L.nin);      // Gaussian init (nn_layer.h:235-239)
            for (int r = 0; r < L.nin; ++r)
                for (int c = 0; c < L.nout; ++c) L.W[(size_t)r * L.nout + c] = T(nd(rng) * std_);
            for (int c = 0; c < L.nout; ++c) L.W[(size_t)L.nin * L.nout + c] = T(0);
            layers.push_back(std::move(L));
        }
        Z.resize(layers.size() + 1);
        F.resize(layers.size() + 1);
        D.resize(layers.size() + 1);
    }

    void ensure(int B) {
        for (size_t l = 0; l <= layers.size(); ++l) {
            const int w = (int)sizes[l] + 1;
            Z[l].resize((size_t)B * w);
            F[l].resize((size_t)B * sizes[l]);
            D[l].resize((size_t)B * sizes[l]);
        }
    }

    // forward one layer l: Z[l] -> Z[l+1] (hidden: sigmoid, last: softmax into Z[L] without ones col use)
    void forward_layer(size_t l, int B) {
        const LayerT<T>& L = layers[l];
        const int wi = L.nin + 1, wo = L.nout + 1;
        std::vector<T> S((size_t)B * L.nout);
        gemm(B, L.nout, wi, Z[l].data(), wi, false, L.W.data(), L.nout, false, S.data(), L.nout, false);
        const bool last = l + 1 == layers.size();
        for (int b = 0; b < B; ++b) {
            T* z = Z[l + 1].data() + (size_t)b * wo;
            const T* s = S.data() + (size_t)b * L.nout;
            if (!last) {
                T* f = F[l + 1].data() + (size_t)b * L.nout;
                for (int j = 0; j < L.nout; ++j) {
                    const T y = T(1) / (T(1) + std::exp(-s[j]));
                    z[j] = y;
                    f[j] = y * (T(1) - y);
                }
            } else {
                T m = s[0];
                for (int j = 1; j < L.nout; ++j) m = std::max(m, s[j]);
                T sum = 0;
                for (int j = 0; j < L.nout; ++j) { z[j] = std::exp(s[j] - m); sum += z[j]; }
                for (int j = 0; j < L.nout; ++j) z[j] /= sum;
            }
            z[L.nout] = T(1);
        }
    }

    void load_input(const float* x, int B) {
        const int w = sizes[0] + 1;
        for (int b = 0; b < B; ++b) {
            for (int j = 0; j < sizes[0]; ++j) Z[0][(size_t)b * w + j] = T(x[(size_t)b * sizes[0] + j]);
            Z[0][(size_t)b * w + sizes[0]] = T(1);
        }
    }

    float loss_of(const int* y, int B, int* wrong) {
        const int nc = sizes.back(), w = nc + 1;
        double loss = 0;
        int bad = 0;
        for (int b = 0; b < B; ++b) {
            const T* p = Z.back().data() + (size_t)b * w;
            loss -= std::log(std::max((double)p[y[b]], 1e-10));     // LogDot with the 1e-10 bump (util.h:138-144)
            int am = 0;
            for (int j = 1; j < nc; ++j)
                if (p[j] > p[am]) am = j;
            bad += am != y[b];
        }
        if (wrong) *wrong = bad;
        return (float)(loss / B);
    }

    // backward from the output; computes G for every layer; layer callback after each gradient
    template <typename CB>
    void backward(const int* y, int B, CB&& on_grad) {
        const size_t nl = layers.size();
        const int nc = sizes.back();
        T* d = D[nl].data();
        for (int b = 0; b < B; ++b)
            for (int j = 0; j < nc; ++j)
                d[(size_t)b * nc + j] = (Z[nl][(size_t)b * (nc + 1) + j] - (j == y[b] ? T(1) : T(0))) / T(B);
        for (size_t l = nl; l-- > 0;) {
            LayerT<T>& L = layers[l];
            const int wi = L.nin + 1;
            // G = Z[l]^T . D[l+1]
            gemm(wi, L.nout, B, Z[l].data(), wi, true, D[l + 1].data(), L.nout, false, L.G.data(), L.nout, false);
            if (!on_grad(l)) return;   // short-circuit
            if (l > 0) {
                // D[l] = (D[l+1] . W[:-1]^T) * F[l]
                gemm(B, L.nin, L.nout, D[l + 1].data(), L.nout, false, L.W.data(), L.nout, true, D[l].data(),
                     L.nin, false);
                for (size_t i = 0; i < (size_t)B * L.nin; ++i) D[l][i] *= F[l][i];
            }
        }
    }

    float step(const float* x, const int* y, int B) {
        ensure(B);
        load_input(x, B);
        for (size_t l = 0; l < layers.size(); ++l) forward_layer(l, B);
        const float loss = loss_of(y, B, nullptr);
        backward(y, B, [](size_t) { return true; });
        return loss;
    }

    void apply(float lr_scale) {
        for (auto& L : layers)
            for (size_t i = 0; i < L.W.size(); ++i) L.W[i] -= T(lr) * T(lr_scale) * L.G[i];
    }

    float evaluate(const float* x, const int* y, int n, float* err) {
        double loss = 0;
        int wrong = 0;
        const int B = 256;
        for (int o = 0; o < n; o += B) {
            const int b = std::min(B, n - o);
            ensure(b);
            load_input(x + (size_t)o * sizes[0], b);
            for (size_t l = 0; l < layers.size(); ++l) forward_layer(l, b);
            int w = 0;
            loss += loss_of(y + o, b, &w) * b;
            wrong += w;
        }
        if (err) *err = (float)wrong / n;
        return (float)(loss / n);
    }
};

using MLP = MLPT<float>;

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int64_t read_step(void* st) {
    if (pdnn_store_get(st, "step", 60000) != 0 || pdnn_store_last_len(st) != 8) return -2;
    int64_t s;
    pdnn_store_copy_last(st, &s);
    return s;
}

std::string key(const char* p, int64_t a, int b = -1, int c = -1) {
    std::string k = std::string(p) + "/" + std::to_string(a);
    if (b >= 0) k += "/" + std::to_string(b);
    if (c >= 0) k += "/" + std::to_string(c);
    return k;
}

}  // namespace

extern "C" {

RT_API void* pdnn_mlp_create(const int* sizes, int n_sizes, int batch, float lr, uint64_t seed) {
    if (n_sizes < 2) return nullptr;
    return new MLP(sizes, n_sizes, batch, lr, seed);
}
RT_API void pdnn_mlp_destroy(void* h) { delete static_cast<MLP*>(h); }
RT_API int pdnn_mlp_n_layers(void* h) { return (int)static_cast<MLP*>(h)->layers.size(); }
RT_API int64_t pdnn_mlp_layer_size(void* h, int l) { return (int64_t) static_cast<MLP*>(h)->layers[l].W.size(); }
RT_API float* pdnn_mlp_weights(void* h, int l) { return static_cast<MLP*>(h)->layers[l].W.data(); }
RT_API float* pdnn_mlp_grads(void* h, int l) { return static_cast<MLP*>(h)->layers[l].G.data(); }
RT_API float pdnn_mlp_forward_backward(void* h, const float* x, const int* labels, int n) {
    return static_cast<MLP*>(h)->step(x, labels, n);
}
RT_API void pdnn_mlp_apply(void* h, float lr_scale) { static_cast<MLP*>(h)->apply(lr_scale); }
RT_API float pdnn_mlp_loss(void* h, const float* x, const int* labels, int n, float* err) {
    return static_cast<MLP*>(h)->evaluate(x, labels, n, err);
}


}  // extern "C"

namespace {

template <typename M>
int train_single_impl(M& m, const float* x, const int* labels, int n, int iters, float* losses) {
    const int B = m.batch, d = m.sizes[0];
    int off = 0;
    std::vector<float> xb((size_t)B * d);
    std::vector<int> yb(B);
    for (int it = 0; it < iters; ++it) {
        for (int b = 0; b < B; ++b) {      // row-offset epoch wrap (fixes defect D16)
            const int r = (off + b) % n;
            memcpy(xb.data() + (size_t)b * d, x + (size_t)r * d, sizeof(float) * d);
            yb[b] = labels[r];
        }
        off = (off + B) % n;
        const float l = m.step(xb.data(), yb.data(), B);
        m.apply(1.f);
        if (losses) losses[it] = l;
    }
    return iters;
}

int64_t get_i64(void* st, const std::string& k, int64_t timeout_ms, bool* ok) {
    int64_t v = 0;
    *ok = pdnn_store_get(st, k.c_str(), timeout_ms) == 0 && pdnn_store_last_len(st) == 8;
    if (*ok) pdnn_store_copy_last(st, &v);
    return v;
}

template <typename T>
int run_role_impl(const char* role, const char* host, int port, int rank, int n_procs, int n_to_collect, int iters,
                  const float* x, const int* labels, int n, const int* sizes, int n_sizes, int batch, float lr,
                  int shortcircuit, const char* out_prefix) {
    void* st = pdnn_store_connect(host, port, 30000);
    if (!st) return -1;
    MLPT<T> m(sizes, n_sizes, batch, lr, 1234);
    const int L = (int)m.layers.size();
    const int n_workers = n_procs - 2;
    std::string r(role);
    const std::string scheme = "SyncReplicasWithBackup" + std::to_string(n_to_collect) + "_" +
                               std::to_string(n_workers) + (shortcircuit ? "_shortcircuit" : "") +
                               (sizeof(T) == 8 ? "_fp64" : "");
    int rc = 0;
    if (r == "master") {
        pdnn_store_set(st, "scheme", scheme.data(), scheme.size());
        void* ps = pdnn_ps_create(n_workers, L, n_to_collect, 0);
        std::string tl = std::string(out_prefix) + "timeline_out_" + scheme;
        FILE* tf = fopen(tl.c_str(), "w");
        const double t0 = now_ms();
        std::vector<std::vector<T>> acc(L);
        std::vector<T> g;
        int64_t qpos = 0;
        for (int64_t s = 1; s <= iters; ++s) {
            pdnn_ps_begin_step(ps, s);
            for (int l = 0; l < L; ++l) {
                auto& W = m.layers[l].W;
                pdnn_store_set(st, key("w", s, l).c_str(), W.data(), W.size() * sizeof(T));
                acc[l].assign(W.size(), T(0));
            }
            pdnn_store_set(st, "step", &s, 8);
            pdnn_store_set(st, key("go", s).c_str(), &s, 8);
            if (tf) fprintf(tf, "%.3f %lld 1\n", now_ms() - t0, (long long)s);
            while (!pdnn_ps_done(ps)) {
                // block on the next announced gradient (MPI_Waitany over the pre-posted receives)
                const std::string qk = key("gq", qpos + 1);
                if (pdnn_store_get(st, qk.c_str(), 60000) != 0) { rc = -4; break; }
                std::string ent(pdnn_store_last_len(st), '\0');
                pdnn_store_copy_last(st, &ent[0]);
                ++qpos;
                pdnn_store_del(st, qk.c_str());
                long long gs = 0;
                int gl = 0, gw = 0;
                if (sscanf(ent.c_str(), "%lld %d %d", &gs, &gl, &gw) != 3) continue;
                const std::string gk = key("g", gs, gl, gw);
                if (gs == s && pdnn_store_get(st, gk.c_str(), 1000) == 0 &&
                    pdnn_store_last_len(st) == acc[gl].size() * sizeof(T)) {
                    g.resize(acc[gl].size());
                    pdnn_store_copy_last(st, g.data());
                    if (pdnn_ps_offer(ps, gw - 2, gl, gs, now_ms() - t0) == 0) {
                        for (size_t i = 0; i < g.size(); ++i) acc[gl][i] += g[i];
                        if (tf) fprintf(tf, "%.3f %lld 0 %d %d\n", now_ms() - t0, (long long)s, gw, gl);
                    }
                } else {
                    pdnn_ps_offer(ps, gw - 2, gl, gs, now_ms() - t0);   // an older step: counted stale, dropped
                }
                pdnn_store_del(st, gk.c_str());
            }
            if (rc) break;
            for (int l = 0; l < L; ++l) {      // ApplyGrad(lr / count): count-correct average fused in
                const int cnt = std::max(1, pdnn_ps_count(ps, l));
                auto& W = m.layers[l].W;
                for (size_t i = 0; i < W.size(); ++i) W[i] -= T(lr) / T(cnt) * acc[l][i];
                if (s > 2) pdnn_store_del(st, key("w", s - 2, l).c_str());
            }
            if (s > 2) pdnn_store_del(st, key("go", s - 2).c_str());
        }
        int64_t stop = -1;
        // publish the final weights as step iters+1 so the evaluator can score the final model
        const int64_t fin = iters + 1;
        for (int l = 0; l < L; ++l)
            pdnn_store_set(st, key("w", fin, l).c_str(), m.layers[l].W.data(), m.layers[l].W.size() * sizeof(T));
        pdnn_store_set(st, "final_step", &fin, 8);
        pdnn_store_set(st, "step", &stop, 8);
        pdnn_store_set(st, key("go", fin).c_str(), &stop, 8);
        // late gradients of the last step(s): drain what is already announced (workers stop at go/<fin>)
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        for (;;) {
            const std::string qk = key("gq", qpos + 1);
            if (pdnn_store_get(st, qk.c_str(), 200) != 0) break;
            std::string ent(pdnn_store_last_len(st), '\0');
            pdnn_store_copy_last(st, &ent[0]);
            ++qpos;
            pdnn_store_del(st, qk.c_str());
            long long gs = 0;
            int gl = 0, gw = 0;
            if (sscanf(ent.c_str(), "%lld %d %d", &gs, &gl, &gw) == 3) {
                pdnn_ps_offer(ps, gw - 2, gl, gs, now_ms() - t0);
                pdnn_store_del(st, key("g", gs, gl, gw).c_str());
            }
        }
        if (tf) {
            fprintf(tf, "# stale_dropped %lld leaked_keys %d\n", (long long)pdnn_ps_stale_dropped(ps),
                    pdnn_store_keys(st, "g/"));
            fclose(tf);
        }
        pdnn_ps_destroy(ps);
    } else if (r == "worker") {
        const int B = batch, d = sizes[0];
        std::vector<float> xb((size_t)B * d);
        std::vector<int> yb(B);
        int off = ((rank - 2) * B) % n;
        int64_t cur = 0;
        for (;;) {
            // a worker that fell behind jumps straight to the newest step (its go/ key may be deleted already);
            // otherwise it blocks until the next step opens (C-08)
            int64_t latest = read_step(st);
            if (latest == -1 || latest == -2) break;
            if (latest <= cur) {
                bool ok = false;
                const int64_t s = get_i64(st, key("go", cur + 1), 120000, &ok);
                if (!ok || s < 0) break;
                latest = std::max(s, read_step(st));
                if (latest < 0) break;
            }
            cur = latest;
            for (int b = 0; b < B; ++b) {
                const int rr = (off + b) % n;
                memcpy(xb.data() + (size_t)b * d, x + (size_t)rr * d, sizeof(float) * d);
                yb[b] = labels[rr];
            }
            off = (off + B * n_workers) % n;
            m.ensure(B);
            m.load_input(xb.data(), B);
            bool abandoned = false;
            auto newer = [&] {
                if (!shortcircuit) return false;
                int64_t now = read_step(st);
                return now != cur;
            };
            for (int l = 0; l < L && !abandoned; ++l) {     // layer-pipelined forward
                if (newer()) { abandoned = true; break; }
                if (pdnn_store_get(st, key("w", cur, l).c_str(), 30000) != 0) { abandoned = true; break; }
                pdnn_store_copy_last(st, m.layers[l].W.data());
                m.forward_layer((size_t)l, B);
            }
            if (abandoned) continue;
            m.backward(yb.data(), B, [&](size_t l) {
                if (newer()) return false;
                const auto& G = m.layers[l].G;
                pdnn_store_set(st, key("g", cur, (int)l, rank).c_str(), G.data(), G.size() * sizeof(T));
                // announce it on the master's arrival queue (tagged with the step: stale-drop key)
                const int64_t q = pdnn_store_add(st, "gq_n", 1);
                const std::string ent = std::to_string(cur) + " " + std::to_string(l) + " " + std::to_string(rank);
                pdnn_store_set(st, key("gq", q).c_str(), ent.data(), ent.size());
                return true;
            });
        }
    } else if (r == "evaluator") {
        if (pdnn_store_get(st, "scheme", 60000) != 0) { pdnn_store_close(st); return -2; }
        std::string sch(pdnn_store_last_len(st), '\0');
        pdnn_store_copy_last(st, &sch[0]);
        std::string fn = std::string(out_prefix) + "time_loss_out_" + sch;
        FILE* f = fopen(fn.c_str(), "w");
        const double t0 = now_ms();
        auto eval_step = [&](int64_t s) {
            for (int l = 0; l < L; ++l) {
                if (pdnn_store_get(st, key("w", s, l).c_str(), 2000) != 0) return;
                pdnn_store_copy_last(st, m.layers[l].W.data());
            }
            float err;
            const float loss = m.evaluate(x, labels, n, &err);
            if (f) { fprintf(f, "%lld %.3f %.6f %.6f\n", (long long)s, now_ms() - t0, loss, err); fflush(f); }
        };
        int64_t next = 1;
        for (;;) {
            int64_t s = pdnn_store_check(st, "step") == 1 ? read_step(st) : 0;
            if (s != -1 && s < next) {
                bool ok = false;
                s = get_i64(st, key("go", next), 120000, &ok);               // blocking: no polling
                if (!ok) break;
            }
            if (s == -1) {
                if (pdnn_store_get(st, "final_step", 2000) == 0) {
                    int64_t fs;
                    pdnn_store_copy_last(st, &fs);
                    eval_step(fs);
                }
                break;
            }
            // skip to the newest step if training ran ahead of the evaluation
            const int64_t latest = read_step(st);
            const int64_t use = latest > s ? latest : s;
            eval_step(use);
            next = use + 1;
        }
        if (f) fclose(f);
    } else {
        rc = -3;
    }
    pdnn_store_close(st);
    return rc;
}

}  // namespace

extern "C" {
// Single-machine training (CPP-11 test_nn / nn.h:53-65): epoch-wrapping batches, returns iterations run.
RT_API int pdnn_mlp_train_single(void* h, const float* x, const int* labels, int n, int iters, float* losses) {
    return train_single_impl(*static_cast<MLP*>(h), x, labels, n, iters, losses);
}

// Same in the reference's fp64 (cblas_dgemm) arithmetic when fp64 != 0; the final full-set loss and error rate
// go to *final_loss / *final_err.
RT_API int pdnn_mlp_train_single_ex(const int* sizes, int n_sizes, int batch, float lr, uint64_t seed,
                                    const float* x, const int* labels, int n, int iters, float* losses, int fp64,
                                    float* final_loss, float* final_err) {
    if (fp64) {
        MLPT<double> m(sizes, n_sizes, batch, lr, seed);
        train_single_impl(m, x, labels, n, iters, losses);
        if (final_loss) *final_loss = m.evaluate(x, labels, n, final_err);
    } else {
        MLPT<float> m(sizes, n_sizes, batch, lr, seed);
        train_single_impl(m, x, labels, n, iters, losses);
        if (final_loss) *final_loss = m.evaluate(x, labels, n, final_err);
    }
    return iters;
}

// role: "master" | "worker" | "evaluator".  rank 0 = master, 1 = evaluator, >= 2 workers (CPP-01).
// Returns 0 on success.  Master writes <out_prefix>timeline_out_<scheme> (ending with a "# stale_dropped N
// leaked_keys K" summary line); evaluator writes <out_prefix>time_loss_out_<scheme>.
RT_API int pdnn_mlp_run_role_ex(const char* role, const char* host, int port, int rank, int n_procs,
                                int n_to_collect, int iters, const float* x, const int* labels, int n,
                                const int* sizes, int n_sizes, int batch, float lr, int shortcircuit,
                                const char* out_prefix, int fp64) {
    if (fp64)
        return run_role_impl<double>(role, host, port, rank, n_procs, n_to_collect, iters, x, labels, n, sizes,
                                     n_sizes, batch, lr, shortcircuit, out_prefix);
    return run_role_impl<float>(role, host, port, rank, n_procs, n_to_collect, iters, x, labels, n, sizes, n_sizes,
                                batch, lr, shortcircuit, out_prefix);
}

RT_API int pdnn_mlp_run_role(const char* role, const char* host, int port, int rank, int n_procs, int n_to_collect,
                             int iters, const float* x, const int* labels, int n, const int* sizes, int n_sizes,
                             int batch, float lr, int shortcircuit, const char* out_prefix) {
    return pdnn_mlp_run_role_ex(role, host, port, rank, n_procs, n_to_collect, iters, x, labels, n, sizes, n_sizes,
                                batch, lr, shortcircuit, out_prefix, 0);
}
}  // extern "C"
