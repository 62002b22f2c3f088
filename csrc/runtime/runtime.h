// Host runtime of pytorch_distributed_nn_amd (CPU-only C++17; no GPU dependency).
//
//   tcp_store.cpp       control-plane key/value store (server + client)
//   ps_coordinator.cpp  parameter-server gradient-collection state machine (k-of-n kill, backup
//                       workers with stale-by-step drop, arrival timeline)
//   idx_reader.cpp      MNIST IDX reader (+ normalise, one-hot, shuffle)
//   mlp_native.cpp      native MLP trainer (bias-folded dense layers, sigmoid/softmax, SGD) with a
//                       single-machine driver and master / worker / evaluator roles over the store
//
// Everything is exported as a flat C API (RT_API) for ctypes and for the `pdnn_mlp` CLI binary.
#pragma once
#include <cstddef>
#include <cstdint>

#define RT_API __attribute__((visibility("default")))

extern "C" {
// ---- tcp store
RT_API void* pdnn_store_server_start(int port);
RT_API int pdnn_store_server_port(void* h);
RT_API void pdnn_store_server_stop(void* h);
RT_API void* pdnn_store_connect(const char* host, int port, int timeout_ms);
RT_API void pdnn_store_close(void* h);
RT_API int pdnn_store_set(void* h, const char* key, const void* val, uint64_t n);
RT_API int pdnn_store_get(void* h, const char* key, int64_t timeout_ms);
RT_API int pdnn_store_wait(void* h, const char* key, int64_t timeout_ms);
RT_API int64_t pdnn_store_add(void* h, const char* key, int64_t delta);
RT_API int64_t pdnn_store_push(void* h, const char* queue, const void* val, uint64_t n);
RT_API int pdnn_store_check(void* h, const char* key);
RT_API int pdnn_store_del(void* h, const char* key);
RT_API int pdnn_store_keys(void* h, const char* prefix);
RT_API uint64_t pdnn_store_last_len(void* h);
RT_API void pdnn_store_copy_last(void* h, void* dst);

// ---- PS coordinator
RT_API void* pdnn_ps_create(int n_workers, int n_layers, int n_to_collect, int kill_k);
RT_API void pdnn_ps_destroy(void* h);
RT_API void pdnn_ps_begin_step(void* h, int64_t step);
RT_API int pdnn_ps_offer(void* h, int worker, int layer, int64_t step, double t_ms);
RT_API int pdnn_ps_done(void* h);
RT_API int pdnn_ps_count(void* h, int layer);
RT_API int pdnn_ps_stragglers(void* h, int sentinel_layer, int* out);
RT_API int pdnn_ps_contributed(void* h, int layer, int worker);
RT_API int64_t pdnn_ps_stale_dropped(void* h);
RT_API int pdnn_ps_timeline(void* h, double* t, int64_t* step, int* worker, int* layer, int cap);

// ---- IDX reader
RT_API int pdnn_idx_read(const char* path, uint8_t* out, int64_t cap, int* dims, int* ndim);
RT_API int pdnn_idx_write(const char* path, const uint8_t* data, const int* dims, int ndim, int magic_type);
RT_API void pdnn_shuffle_indices(int64_t* idx, int64_t n, uint64_t seed);

// ---- native MLP
RT_API void* pdnn_mlp_create(const int* sizes, int n_sizes, int batch, float lr, uint64_t seed);
RT_API void pdnn_mlp_destroy(void* h);
RT_API int pdnn_mlp_n_layers(void* h);
RT_API int64_t pdnn_mlp_layer_size(void* h, int layer);
RT_API float* pdnn_mlp_weights(void* h, int layer);
RT_API float* pdnn_mlp_grads(void* h, int layer);
RT_API float pdnn_mlp_forward_backward(void* h, const float* x, const int* labels, int n);
RT_API void pdnn_mlp_apply(void* h, float lr_scale);
RT_API float pdnn_mlp_loss(void* h, const float* x, const int* labels, int n, float* err_rate);
RT_API int pdnn_mlp_train_single(void* h, const float* x, const int* labels, int n, int iters, float* losses);
RT_API int pdnn_mlp_run_role(const char* role, const char* host, int port, int rank, int n_procs,
                             int n_to_collect, int iters, const float* x, const int* labels, int n,
                             const int* sizes, int n_sizes, int batch, float lr, int shortcircuit,
                             const char* out_prefix);
// fp64 != 0: the reference's double-precision arithmetic (MPI_code/src/util/util.h:35-81 cblas_dgemm)
RT_API int pdnn_mlp_run_role_ex(const char* role, const char* host, int port, int rank, int n_procs,
                                int n_to_collect, int iters, const float* x, const int* labels, int n,
                                const int* sizes, int n_sizes, int batch, float lr, int shortcircuit,
                                const char* out_prefix, int fp64);
RT_API int pdnn_mlp_train_single_ex(const int* sizes, int n_sizes, int batch, float lr, uint64_t seed,
                                    const float* x, const int* labels, int n, int iters, float* losses, int fp64,
                                    float* final_loss, float* final_err);
}
