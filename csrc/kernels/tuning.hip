// The dispatch table of tuning.h: defaults, the PDNN_TUNE override string and the C API.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.h"
#include "tuning.h"

namespace pg {
namespace {
std::string g_tune_error;

int* field(Tune& t, const char* name) {
#define PDNN_TUNE_LOOKUP(n, d, doc) if (!strcmp(name, #n)) return &t.n;
    PDNN_TUNE_TABLE(PDNN_TUNE_LOOKUP)
#undef PDNN_TUNE_LOOKUP
    return nullptr;
}

// keys of PDNN_TUNE that are not in this table: the Python side checks them against ITS table
// (pytorch_distributed_nn_amd/tuning.py), so neither side keeps a copy of the other's key list
std::string g_tune_unknown;

Tune make() {
    Tune t;
    const char* e = getenv("PDNN_TUNE");
    if (!e) return t;
    std::string s(e);
    size_t pos = 0;
    while (pos <= s.size()) {
        size_t c = s.find(',', pos);
        if (c == std::string::npos) c = s.size();
        const std::string item = s.substr(pos, c - pos);
        pos = c + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        const std::string k = item.substr(0, eq);
        if (eq == std::string::npos) { g_tune_error += "PDNN_TUNE: '" + item + "' is not key=value; "; continue; }
        int* f = field(t, k.c_str());
        if (f) *f = atoi(item.c_str() + eq + 1);
        else g_tune_unknown += (g_tune_unknown.empty() ? "" : ",") + k;
    }
    return t;
}
}  // namespace

Tune& tune() {
    static Tune t = make();
    return t;
}

namespace {
int g_comm_world = 1;
}

int grid_cus() {
    static int hw = 0;
    if (!hw) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&hw, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || hw <= 0) hw = 256;
    }
    int n = hw;
    if (g_comm_world > 1 && tune().comm_cus > 0) n -= tune().comm_cus;
    n = (n / 8) * 8;
    return n < 8 ? 8 : n;
}

}  // namespace pg

// old value, or INT32_MIN for an unknown name
PDNN_API int pdnn_tune_set(const char* name, int value) {
    int* f = pg::field(pg::tune(), name);
    if (!f) return (int)0x80000000;
    const int old = *f;
    *f = value;
    return old;
}

// world size of the process group the caller's collectives run on (1 = no concurrent RCCL kernels to make room
// for); returns the previous value
PDNN_API int pdnn_set_comm_world(int world) {
    const int old = pg::g_comm_world;
    pg::g_comm_world = world < 1 ? 1 : world;
    return old;
}

PDNN_API int pdnn_grid_cus() { return pg::grid_cus(); }

PDNN_API int pdnn_tune_get(const char* name) {
    int* f = pg::field(pg::tune(), name);
    return f ? *f : (int)0x80000000;
}

// "name=value|default|doc\n" per entry into buf (truncated to n bytes); returns the full length
PDNN_API int pdnn_tune_list(char* buf, int n) {
    std::string out;
    const pg::Tune& t = pg::tune();
#define PDNN_TUNE_LIST(nm, d, doc) out += std::string(#nm) + "=" + std::to_string(t.nm) + "|" + std::to_string(d) + "|" + doc + "\n";
    PDNN_TUNE_TABLE(PDNN_TUNE_LIST)
#undef PDNN_TUNE_LIST
    if (buf && n > 0) {
        strncpy(buf, out.c_str(), n - 1);
        buf[n - 1] = 0;
    }
    return (int)out.size();
}

// empty when PDNN_TUNE parsed cleanly
PDNN_API const char* pdnn_tune_error() {
    pg::tune();
    return pg::g_tune_error.c_str();
}

// comma-separated PDNN_TUNE keys this (kernel-side) table does not have
PDNN_API const char* pdnn_tune_unknown() {
    pg::tune();
    return pg::g_tune_unknown.c_str();
}
