// Control-plane key/value store over TCP (SURVEY.md §2.7 / §5.8 "control plane").
//
// Replaces the reference's side channels: the step broadcast (MPI tag 10 / tag 0:
// pytorch_code/sync_replicas_master_nn.py:235-241, MPI_code/.../sync_replicas_master_nn.h:155-161),
// the kill token (tag 77: sync_replicas_master_nn.py:309-314), the evaluator's scheme-name message
// (sync_replicas_master_nn.h:151-153) and the Twisted PB timing RPC (distributed_TF/src/timeout_manager.py).
// Data-plane tensors never go through it: those are RCCL collectives.
//
// Protocol (little endian): request  = u8 op | u32 klen | key | u64 vlen | value
//                           response = u8 status | u64 len | data
// ops: SET, GET (blocking up to timeout_ms carried in value), ADD (int64 delta -> new value),
//      CHECK (exists?), DEL, WAIT (block until key exists), KEYS (newline-joined keys with prefix),
//      PUSH (append to a queue in ONE round trip: n = ++<key>_n, <key>/<n> = value -> n; the arrival queue of
//      the parameter server, whose workers used to pay an ADD and a SET per gradient bucket)
// One server thread per connection; waits are condition-variable based (no polling).
#include "runtime.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {
constexpr uint32_t kMaxKey = 1u << 20;            // 1 MiB keys
constexpr uint64_t kMaxValue = 1ull << 30;        // 1 GiB values (the native MLP moves weight blobs)
}  // namespace

namespace {

enum Op : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, DEL = 5, WAIT = 6, KEYS = 7, PING = 8, PUSH = 9 };
enum Status : uint8_t { OK = 0, TIMEOUT = 1, MISSING = 2, ERR = 3 };

bool send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}
bool recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        ssize_t k = ::recv(fd, c, n, 0);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

struct Server {
    int lfd = -1;
    int port = 0;
    std::atomic<bool> stop{false};
    std::thread acceptor;
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::string, std::vector<char>> kv;
    std::vector<std::thread> workers;
    std::vector<int> fds;

    void reply(int fd, uint8_t st, const void* d, uint64_t n) {
        send_all(fd, &st, 1);
        send_all(fd, &n, 8);
        if (n) send_all(fd, d, n);
    }

    void serve(int fd) {
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        for (;;) {
            uint8_t op;
            uint32_t kl;
            uint64_t vl;
            if (!recv_all(fd, &op, 1) || !recv_all(fd, &kl, 4)) break;
            // lengths come from the wire: a stray or malformed peer must not make the detached serve
            // thread throw bad_alloc (std::terminate would take the whole master down) -> drop it
            if (kl > kMaxKey) break;
            std::string key(kl, '\0');
            if (kl && !recv_all(fd, &key[0], kl)) break;
            if (!recv_all(fd, &vl, 8) || vl > kMaxValue) break;
            std::vector<char> val(vl);
            if (vl && !recv_all(fd, val.data(), vl)) break;
            if (op == SET) {
                {
                    std::lock_guard<std::mutex> g(mu);
                    kv[key] = std::move(val);
                }
                cv.notify_all();
                reply(fd, OK, nullptr, 0);
            } else if (op == GET || op == WAIT) {
                int64_t tmo = -1;
                if (vl >= 8) memcpy(&tmo, val.data(), 8);
                std::unique_lock<std::mutex> lk(mu);
                auto pred = [&] { return stop.load() || kv.count(key) > 0; };
                bool ok;
                if (tmo < 0) { cv.wait(lk, pred); ok = kv.count(key) > 0; }
                // system_clock deadline: pthread_cond_timedwait (libstdc++'s steady_clock wait_for uses
                // pthread_cond_clockwait, which this toolchain's ThreadSanitizer cannot see through)
                else ok = cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(tmo), pred) &&
                          kv.count(key) > 0;
                if (!ok) { lk.unlock(); reply(fd, TIMEOUT, nullptr, 0); continue; }
                if (op == WAIT) { lk.unlock(); reply(fd, OK, nullptr, 0); continue; }
                std::vector<char> out = kv[key];
                lk.unlock();
                reply(fd, OK, out.data(), out.size());
            } else if (op == ADD) {
                int64_t d = 0, nv;
                if (vl >= 8) memcpy(&d, val.data(), 8);
                {
                    std::lock_guard<std::mutex> g(mu);
                    auto& v = kv[key];
                    int64_t cur = 0;
                    if (v.size() == 8) memcpy(&cur, v.data(), 8);
                    nv = cur + d;
                    v.resize(8);
                    memcpy(v.data(), &nv, 8);
                }
                cv.notify_all();
                reply(fd, OK, &nv, 8);
            } else if (op == CHECK) {
                uint8_t e;
                {
                    std::lock_guard<std::mutex> g(mu);
                    e = kv.count(key) ? 1 : 0;
                }
                reply(fd, OK, &e, 1);
            } else if (op == DEL) {
                {
                    std::lock_guard<std::mutex> g(mu);
                    kv.erase(key);
                }
                reply(fd, OK, nullptr, 0);
            } else if (op == KEYS) {
                std::string out;
                {
                    std::lock_guard<std::mutex> g(mu);
                    for (auto it = kv.lower_bound(key); it != kv.end() && it->first.compare(0, key.size(), key) == 0; ++it) {
                        out += it->first;
                        out += '\n';
                    }
                }
                reply(fd, OK, out.data(), out.size());
            } else if (op == PUSH) {
                int64_t nv;
                {
                    std::lock_guard<std::mutex> g(mu);
                    auto& c = kv[key + "_n"];
                    int64_t cur = 0;
                    if (c.size() == 8) memcpy(&cur, c.data(), 8);
                    nv = cur + 1;
                    c.resize(8);
                    memcpy(c.data(), &nv, 8);
                    kv[key + "/" + std::to_string(nv)] = std::move(val);
                }
                cv.notify_all();
                reply(fd, OK, &nv, 8);
            } else if (op == PING) {
                reply(fd, OK, nullptr, 0);
            } else {
                reply(fd, ERR, nullptr, 0);
            }
        }
        ::close(fd);
    }

    bool start(int want_port) {
        lfd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (lfd < 0) return false;
        int one = 1;
        setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_ANY);
        a.sin_port = htons((uint16_t)want_port);
        if (::bind(lfd, (sockaddr*)&a, sizeof(a)) < 0 || ::listen(lfd, 128) < 0) {
            ::close(lfd);
            return false;
        }
        socklen_t len = sizeof(a);
        getsockname(lfd, (sockaddr*)&a, &len);
        port = ntohs(a.sin_port);
        acceptor = std::thread([this] {
            for (;;) {
                int fd = ::accept(lfd, nullptr, nullptr);
                if (fd < 0) {
                    if (stop.load()) break;
                    continue;
                }
                std::lock_guard<std::mutex> g(mu);
                fds.push_back(fd);
                workers.emplace_back([this, fd] { serve(fd); });
            }
        });
        return true;
    }

    void shutdown() {
        stop.store(true);
        cv.notify_all();
        ::shutdown(lfd, SHUT_RDWR);
        ::close(lfd);
        if (acceptor.joinable()) acceptor.join();
        {
            std::lock_guard<std::mutex> g(mu);
            for (int fd : fds) ::shutdown(fd, SHUT_RDWR);
        }
        for (auto& t : workers)
            if (t.joinable()) t.join();
    }
};

struct Client {
    int fd = -1;
    std::mutex mu;
    std::vector<char> last;

    bool connect_to(const char* host, int port, int timeout_ms) {
        auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
        for (;;) {
            addrinfo hints{}, *res = nullptr;
            hints.ai_family = AF_INET;
            hints.ai_socktype = SOCK_STREAM;
            std::string ps = std::to_string(port);
            if (getaddrinfo(host, ps.c_str(), &hints, &res) == 0) {
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
                    freeaddrinfo(res);
                    int one = 1;
                    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                    return true;
                }
                if (fd >= 0) ::close(fd);
                fd = -1;
                freeaddrinfo(res);
            }
            if (std::chrono::steady_clock::now() > deadline) return false;
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
    }

    // returns status, response in `last`; with `out` the response is also copied out while the handle's
    // lock is still held, so one handle may be shared by threads for the single-call ops (add / check)
    int rpc(uint8_t op, const std::string& key, const void* val, uint64_t vl, std::vector<char>* out = nullptr) {
        std::lock_guard<std::mutex> g(mu);
        uint32_t kl = (uint32_t)key.size();
        if (!send_all(fd, &op, 1) || !send_all(fd, &kl, 4) || (kl && !send_all(fd, key.data(), kl)) ||
            !send_all(fd, &vl, 8) || (vl && !send_all(fd, val, vl)))
            return -1;
        uint8_t st;
        uint64_t n;
        if (!recv_all(fd, &st, 1) || !recv_all(fd, &n, 8)) return -1;
        last.resize(n);
        if (n && !recv_all(fd, last.data(), n)) return -1;
        if (out) *out = last;
        return st;
    }
};

}  // namespace

extern "C" {

RT_API void* pdnn_store_server_start(int port) {
    auto* s = new Server();
    if (!s->start(port)) {
        delete s;
        return nullptr;
    }
    return s;
}
RT_API int pdnn_store_server_port(void* h) { return static_cast<Server*>(h)->port; }
RT_API void pdnn_store_server_stop(void* h) {
    auto* s = static_cast<Server*>(h);
    s->shutdown();
    delete s;
}

RT_API void* pdnn_store_connect(const char* host, int port, int timeout_ms) {
    auto* c = new Client();
    if (!c->connect_to(host, port, timeout_ms)) {
        delete c;
        return nullptr;
    }
    return c;
}
RT_API void pdnn_store_close(void* h) {
    auto* c = static_cast<Client*>(h);
    if (c->fd >= 0) ::close(c->fd);
    delete c;
}
RT_API int pdnn_store_set(void* h, const char* key, const void* val, uint64_t n) {
    return static_cast<Client*>(h)->rpc(SET, key, val, n);
}
// Blocking get with timeout (ms, <0 = forever).  Returns status; the value is fetched with
// pdnn_store_last (len) + pdnn_store_copy_last.
RT_API int pdnn_store_get(void* h, const char* key, int64_t timeout_ms) {
    return static_cast<Client*>(h)->rpc(GET, key, &timeout_ms, 8);
}
RT_API int pdnn_store_wait(void* h, const char* key, int64_t timeout_ms) {
    return static_cast<Client*>(h)->rpc(WAIT, key, &timeout_ms, 8);
}
RT_API int64_t pdnn_store_add(void* h, const char* key, int64_t delta) {
    auto* c = static_cast<Client*>(h);
    std::vector<char> r;
    if (c->rpc(ADD, key, &delta, 8, &r) != 0 || r.size() != 8) return INT64_MIN;
    int64_t v;
    memcpy(&v, r.data(), 8);
    return v;
}
RT_API int64_t pdnn_store_push(void* h, const char* queue, const void* val, uint64_t n) {
    auto* c = static_cast<Client*>(h);
    std::vector<char> r;
    if (c->rpc(PUSH, queue, val, n, &r) != 0 || r.size() != 8) return INT64_MIN;
    int64_t v;
    memcpy(&v, r.data(), 8);
    return v;
}
RT_API int pdnn_store_check(void* h, const char* key) {
    auto* c = static_cast<Client*>(h);
    std::vector<char> r;
    if (c->rpc(CHECK, key, nullptr, 0, &r) != 0 || r.empty()) return -1;
    return r[0];
}
RT_API int pdnn_store_del(void* h, const char* key) { return static_cast<Client*>(h)->rpc(DEL, key, nullptr, 0); }
RT_API int pdnn_store_keys(void* h, const char* prefix) { return static_cast<Client*>(h)->rpc(KEYS, prefix, nullptr, 0); }
RT_API uint64_t pdnn_store_last_len(void* h) { return static_cast<Client*>(h)->last.size(); }
RT_API void pdnn_store_copy_last(void* h, void* dst) {
    auto* c = static_cast<Client*>(h);
    if (!c->last.empty()) memcpy(dst, c->last.data(), c->last.size());
}

}  // extern "C"
