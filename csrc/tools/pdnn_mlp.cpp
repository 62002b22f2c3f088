// pdnn_mlp — command-line driver of the native (C++) MLP stack (CPP-01 distributed
// driver, CPP-11 single-machine test binary, CPP-12 build/run targets; reference: MPI_code/src/
// distributed_nn.cpp:16-86, single_machine_nn.cpp:5-12, Makefile:1-19).
//
// The reference runs one MPI rank per process (`mpirun -n 8 ./distributed_nn`).  Here the control
// plane is the framework's TCP store (csrc/runtime/tcp_store.cpp) and the ranks are plain processes:
//
//   pdnn_mlp single      [--data DIR] [--iters N] [--batch B] [--lr LR] [--fp64]
//   pdnn_mlp distributed [--nprocs 8] [--collect K] [--iters N] [--data DIR] [--shortcircuit] [--fp64] [--out PREFIX]
//                        (forks master + evaluator + nprocs-2 workers around a local store: `make distributed_run`)
//   pdnn_mlp store       --port P                       (stand-alone store server for multi-host runs)
//   pdnn_mlp role        --role master|evaluator|worker --rank R --nprocs N --host H --port P [...]
//
// Model: 784-500-500-800-800-200-100-100-10 sigmoid MLP with softmax output (distributed_nn.cpp:36-47),
// batch 128, lr 1e-3.  Data: MNIST IDX files in --data, else a deterministic synthetic MNIST-shaped set.
#include <sys/wait.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "runtime.h"

namespace {

struct Args {
    std::string cmd, data, role = "worker", host = "127.0.0.1", out = "";
    int iters = 100, batch = 128, nprocs = 8, collect = 0, rank = 0, port = 0, shortcircuit = 0, fp64 = 0;
    float lr = 1e-3f;
};

const std::vector<int> kSizes = {784, 500, 500, 800, 800, 200, 100, 100, 10};

bool load_mnist(const std::string& dir, std::vector<float>& x, std::vector<int>& y) {
    int dims[4], nd = 0;
    const std::string fi = dir + "/train-images-idx3-ubyte", fl = dir + "/train-labels-idx1-ubyte";
    if (pdnn_idx_read(fi.c_str(), nullptr, 0, dims, &nd) != -4 || nd != 3) return false;
    const int64_t n = dims[0], d = (int64_t)dims[1] * dims[2];
    std::vector<uint8_t> img(n * d), lab(n);
    if (pdnn_idx_read(fi.c_str(), img.data(), img.size(), dims, &nd) != (int)img.size()) return false;
    if (pdnn_idx_read(fl.c_str(), lab.data(), lab.size(), dims, &nd) != (int)lab.size()) return false;
    x.resize(n * d);
    y.resize(n);
    for (int64_t i = 0; i < n * d; ++i) x[i] = img[i] / 255.0f;
    for (int64_t i = 0; i < n; ++i) y[i] = lab[i];
    return true;
}

void synth_mnist(int n, std::vector<float>& x, std::vector<int>& y) {
    // a learnable pattern: a bright column per class over low-amplitude noise (same as data.write_mnist_like)
    x.assign((size_t)n * 784, 0.f);
    y.resize(n);
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        y[i] = (int)((s >> 33) % 10);
        for (int p = 0; p < 784; ++p) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            x[(size_t)i * 784 + p] = (float)((s >> 40) & 63) / 255.0f;
        }
        for (int r = 4; r < 24; ++r) x[(size_t)i * 784 + r * 28 + 2 + 2 * y[i]] = 1.0f;
    }
}

void get_data(const Args& a, std::vector<float>& x, std::vector<int>& y) {
    if (!a.data.empty() && load_mnist(a.data, x, y)) {
        fprintf(stderr, "pdnn_mlp: loaded %zu MNIST images from %s\n", y.size(), a.data.c_str());
        return;
    }
    synth_mnist(2048, x, y);
    fprintf(stderr, "pdnn_mlp: using %zu synthetic MNIST-shaped images\n", y.size());
}

int run_single(const Args& a) {     // CPP-11: test_load_data(); test_nn();
    std::vector<float> x;
    std::vector<int> y;
    get_data(a, x, y);
    std::vector<float> losses(a.iters);
    float l = 0.f, err = 0.f;
    pdnn_mlp_train_single_ex(kSizes.data(), (int)kSizes.size(), a.batch, a.lr, 1234, x.data(), y.data(),
                             (int)y.size(), a.iters, losses.data(), a.fp64, &l, &err);
    for (int i = 0; i < a.iters; ++i)
        if (i % 10 == 0 || i == a.iters - 1) printf("iter %d loss %.5f\n", i, losses[i]);
    printf("final loss %.5f error rate %.4f (%s)\n", l, err, a.fp64 ? "fp64" : "fp32");
    return std::isfinite(l) ? 0 : 1;
}

int run_role(const Args& a, const std::vector<float>& x, const std::vector<int>& y) {
    return pdnn_mlp_run_role_ex(a.role.c_str(), a.host.c_str(), a.port, a.rank, a.nprocs, a.collect, a.iters,
                                x.data(), y.data(), (int)y.size(), kSizes.data(), (int)kSizes.size(), a.batch, a.lr,
                                a.shortcircuit, a.out.c_str(), a.fp64);
}

int run_distributed(Args a) {       // CPP-12 distributed_run: master (0) + evaluator (1) + workers (2..)
    if (a.nprocs < 3) {
        fprintf(stderr, "pdnn_mlp: --nprocs must be >= 3 (master, evaluator, >= 1 worker)\n");
        return 2;
    }
    if (a.collect <= 0) a.collect = a.nprocs - 2;
    std::vector<float> x;
    std::vector<int> y;
    get_data(a, x, y);
    void* srv = pdnn_store_server_start(a.port);
    if (!srv) return 3;
    a.port = pdnn_store_server_port(srv);
    std::vector<pid_t> kids;
    for (int r = 0; r < a.nprocs; ++r) {
        pid_t pid = fork();
        if (pid == 0) {
            Args b = a;
            b.rank = r;
            b.role = r == 0 ? "master" : (r == 1 ? "evaluator" : "worker");
            _exit(run_role(b, x, y) == 0 ? 0 : 1);
        }
        kids.push_back(pid);
    }
    int bad = 0;
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        bad += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    }
    pdnn_store_server_stop(srv);
    printf("distributed run finished: %d process(es) failed; timelines under '%s'\n", bad, a.out.c_str());
    return bad ? 1 : 0;
}

void usage() {
    fprintf(stderr,
            "usage: pdnn_mlp single|distributed|store|role [--data DIR] [--iters N] [--batch B] [--lr LR]\n"
            "       [--nprocs N] [--collect K] [--shortcircuit] [--fp64] [--out PREFIX] [--role R] [--rank R]\n"
            "       [--host H] [--port P]\n");
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        usage();
        return 2;
    }
    Args a;
    a.cmd = argv[1];
    for (int i = 2; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) { usage(); exit(2); }
            return argv[++i];
        };
        if (k == "--data") a.data = val();
        else if (k == "--iters") a.iters = atoi(val());
        else if (k == "--batch") a.batch = atoi(val());
        else if (k == "--lr") a.lr = (float)atof(val());
        else if (k == "--nprocs") a.nprocs = atoi(val());
        else if (k == "--collect") a.collect = atoi(val());
        else if (k == "--shortcircuit") a.shortcircuit = 1;
        else if (k == "--fp64") a.fp64 = 1;
        else if (k == "--out") a.out = val();
        else if (k == "--role") a.role = val();
        else if (k == "--rank") a.rank = atoi(val());
        else if (k == "--host") a.host = val();
        else if (k == "--port") a.port = atoi(val());
        else { usage(); return 2; }
    }
    if (a.cmd == "single") return run_single(a);
    if (a.cmd == "distributed") return run_distributed(a);
    if (a.cmd == "store") {
        void* srv = pdnn_store_server_start(a.port);
        if (!srv) return 3;
        printf("store listening on port %d\n", pdnn_store_server_port(srv));
        fflush(stdout);
        pause();
        return 0;
    }
    if (a.cmd == "role") {
        std::vector<float> x;
        std::vector<int> y;
        get_data(a, x, y);
        if (a.collect <= 0) a.collect = a.nprocs - 2;
        return run_role(a, x, y);
    }
    usage();
    return 2;
}
