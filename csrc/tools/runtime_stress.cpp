// Concurrency stress of the host runtime for the race detector: built with
// -fsanitize=thread (or address) by tests/test_sanitizers_cpu.py and run on the CPU box.
//
//  * 8 client threads hammer one TCP store server: set / get / atomic add / blocking wait on shared and
//    private keys (the server's per-connection worker threads and its condition-variable waits);
//  * a shared client handle is used from several threads at once (the client's own mutex);
//  * one PS coordinator per thread runs full k-of-n / backup-worker steps (no shared state by design).
// Exit code 0 when every operation returned the expected value; the sanitizer reports races itself.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

int main() {
    void* srv = pdnn_store_server_start(0);
    if (!srv) return 10;
    const int port = pdnn_store_server_port(srv);
    std::atomic<int> errors{0};
    void* shared = pdnn_store_connect("127.0.0.1", port, 5000);
    const int T = 8, N = 200;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
            void* c = pdnn_store_connect("127.0.0.1", port, 5000);
            if (!c) { errors++; return; }
            for (int i = 0; i < N; ++i) {
                const std::string k = "k/" + std::to_string(t) + "/" + std::to_string(i);
                const int64_t v = (int64_t)t * 1000 + i;
                if (pdnn_store_set(c, k.c_str(), &v, sizeof v) != 0) errors++;
                if (pdnn_store_get(c, k.c_str(), 1000) != 0 || pdnn_store_last_len(c) != sizeof v) { errors++; continue; }
                int64_t r = 0;
                pdnn_store_copy_last(c, &r);
                if (r != v) errors++;
                pdnn_store_add(c, "counter", 1);
                pdnn_store_add(shared, "shared_counter", 1);          // one handle, many threads
            }
            // barrier through the store: wait for every thread's last key
            for (int u = 0; u < T; ++u) {
                const std::string k = "k/" + std::to_string(u) + "/" + std::to_string(N - 1);
                if (pdnn_store_wait(c, k.c_str(), 10000) != 0) errors++;
            }
            void* ps = pdnn_ps_create(4, 3, 2, 0);
            for (int s = 1; s <= 20; ++s) {
                pdnn_ps_begin_step(ps, s);
                for (int w = 0; w < 4 && !pdnn_ps_done(ps); ++w)
                    for (int l = 0; l < 3; ++l) pdnn_ps_offer(ps, (w + s) % 4, l, s, 0.0);
                if (!pdnn_ps_done(ps) || pdnn_ps_count(ps, 0) != 2) errors++;
                pdnn_ps_offer(ps, 0, 0, s - 1, 0.0);                   // stale: must be dropped
            }
            pdnn_ps_destroy(ps);
            pdnn_store_close(c);
        });
    }
    for (auto& x : th) x.join();
    if (pdnn_store_add(shared, "counter", 0) != (int64_t)T * N) errors++;
    if (pdnn_store_add(shared, "shared_counter", 0) != (int64_t)T * N) errors++;
    pdnn_store_close(shared);
    pdnn_store_server_stop(srv);
    printf("runtime_stress: %d error(s)\n", errors.load());
    return errors.load() == 0 ? 0 : 1;
}
