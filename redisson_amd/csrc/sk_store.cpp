// sk_store.cpp -- GPU-resident sketch store + batched command executor behind
// the C ABI in include/redisson_sketch.h.
//
// Replaces, for sketch key types, what Redisson's L3 executor hands to Netty
// and redis-server (M:command/CommandAsyncService.java:378, batch hook
// M:command/CommandBatchService.java:91-111,184-293).  Host work here is
// bookkeeping only (key directory, validation, capacity, error text, and the
// final scalar steps of PFCOUNT / Bloom count); every per-element and
// per-register step runs in the HIP kernels of sk_kernels.hip.  There is no
// CPU fallback: without a working device sk_open() fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <rccl/rccl.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/redisson_sketch.h"
#include "sk_internal.h"
#include "sk_hllstr.h"
#include "sk_rdb.h"

using namespace sk_hll;

namespace {

// Host worker threads, started once per process.  The host passes that run on every large call (handle liveness
// checks, directory lookups, estimator tails, staging copies) used to spawn and join up to 16 std::threads per call
// (~20-50 us each); the pool keeps them parked on a condition variable.  run(parts, fn) calls fn(0..parts-1) on the
// workers and the caller and returns when all are done; one parallel section at a time (contexts share the pool).
class HostPool {
  public:
    static HostPool &get() {
        // never destroyed: parked workers end with the process.  A forked child has none of the parent's threads,
        // so it starts its own pool.
        static std::mutex m;
        static HostPool *p = nullptr;
        static pid_t pid = 0;
        std::lock_guard<std::mutex> l(m);
        if (!p || pid != getpid()) {
            p = new HostPool();
            pid = getpid();
        }
        return *p;
    }
    unsigned threads() const { return unsigned(workers_.size()) + 1; }
    // An exception thrown by fn (bad_alloc in a lookup pass ...) is caught where it is thrown, the section still
    // waits until every worker has left fn -- which references the caller's frame -- and then the first exception is
    // rethrown on the caller.  A run() nested inside a section (fn calling host_for) runs inline on the
    // calling thread instead of waiting on run_mu_, which its own section holds.
    void run(unsigned parts, const std::function<void(unsigned)> &fn) {
        if (parts <= 1 || workers_.empty() || in_section()) {
            for (unsigned t = 0; t < parts; t++) fn(t);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> l(mu_);
            job_ = &fn;
            parts_ = parts;
            next_.store(0);
            active_ = unsigned(workers_.size());
            err_ = nullptr;
            gen_++;
        }
        cv_.notify_all();
        in_section() = true;
        work(fn, parts);
        in_section() = false;
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [&] { return active_ == 0; });
        job_ = nullptr;
        std::exception_ptr e = err_;
        err_ = nullptr;
        l.unlock();
        if (e) std::rethrow_exception(e);
    }

  private:
    static bool &in_section() {
        static thread_local bool b = false;
        return b;
    }
    // take parts until none is left; an exception is recorded (first one wins) and the remaining parts are skipped
    void work(const std::function<void(unsigned)> &fn, unsigned P) {
        for (unsigned t; (t = next_.fetch_add(1)) < P;) {
            try {
                fn(t);
            } catch (...) {
                std::lock_guard<std::mutex> l(mu_);
                if (!err_) err_ = std::current_exception();
                next_.store(P);
            }
        }
    }
    HostPool() {
        unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (const char *e = getenv("OMP_NUM_THREADS")) T = std::max(1, std::min(int(T), atoi(e)));
        for (unsigned i = 1; i < T; i++) workers_.emplace_back([this] { loop(); });
        for (auto &w : workers_) w.detach();
    }
    void loop() {
        uint64_t seen = 0;
        in_section() = true; // a worker is only ever inside a section
        for (;;) {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return gen_ != seen; });
            seen = gen_;
            const std::function<void(unsigned)> *j = job_;
            const unsigned P = parts_;
            l.unlock();
            work(*j, P);
            l.lock();
            if (--active_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)> *job_ = nullptr;
    unsigned parts_ = 0, active_ = 0;
    std::atomic<unsigned> next_{0};
    uint64_t gen_ = 0;
    std::exception_ptr err_;
};
// parallel for over [0, n) in `parts` contiguous ranges (parts = the pool's threads unless n is small)
void host_for(uint64_t n, uint64_t min_per_thread, const std::function<void(uint64_t, uint64_t)> &fn) {
    HostPool &p = HostPool::get();
    const unsigned T = n >= 2 * min_per_thread ? unsigned(std::min<uint64_t>(p.threads(), n / min_per_thread)) : 1u;
    if (T <= 1) {
        fn(0, n);
        return;
    }
    p.run(T, [&](unsigned t) { fn(n * t / T, n * (t + 1) / T); });
}

constexpr uint64_t kHllBytes = 16384;   // registers per HLL: the u8 register arrays (host side, union buffers)
constexpr uint64_t kSlabBytes = 12288;  // a slab of the HBM arena: Redis's dense register body (SK_SLAB_BYTES)
constexpr int64_t kBloomMaxSize = 2LL * 2147483647LL; // M:RedissonBloomFilter.java:52
constexpr uint32_t kNoId = 0xffffffffu;

struct DirEnt { // mirrors sk::DirEnt in sk_kernels.hip
    uint8_t *ptr;
    uint64_t len;
    uint64_t cap;
};

struct KeyEnt {
    int type;
    uint32_t id;
};

struct BloomCfg {
    int64_t size;
    int32_t k;
    int64_t expected;
    double fpp;
    sk_rdb::Fields fields; // the hash as stored (HMSET order and value strings), what DUMP / SAVE write
    uint64_t seq = 0;      // its SCAN position: set once when the key is created, unique in the context
};

struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        // large buffers: 1/8 headroom in 2 MiB steps, so batches of slightly varying size do not reallocate (a
        // hipFree synchronises the device and cost 28 ms once with a large keyspace resident); small ones exact on
        // the first allocation, then at least doubling (a slowly growing small request must not free every call)
        size_t nc = cap ? std::max(bytes, cap * 2) : bytes;
        if (bytes >= (size_t(1) << 20)) {
            nc = std::max(bytes + bytes / 8, cap * 2);
            nc = (nc + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
        }
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        hipError_t e = hipMalloc(&p, nc);
        if (e != hipSuccess) return e;
        cap = nc;
        return hipSuccess;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

unsigned bits_for(uint64_t maxval) { // bits needed to represent values 0..maxval
    unsigned b = 0;
    while (b < 64 && (maxval >> b)) b++;
    return b ? b : 1;
}

uint64_t round16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

double g_pe[64];
struct PeInit {
    PeInit() {
        g_pe[0] = 1;
        for (int j = 1; j < 64; j++) g_pe[j] = 1.0 / double(1ULL << j);
    }
} g_pe_init;

// ---- estimator (redis hyperloglog.c hllCount) -------------------------
uint64_t estimate_v3(double E, int ez) {
    const double m = 16384;
    double alpha = 0.7213 / (1 + 1.079 / m);
    E = (1 / E) * alpha * m * m;
    if (E < m * 2.5 && ez != 0) {
        E = m * std::log(m / ez);
    } else if (E < 72000) { // m == 16384
        double bias = 5.9119 * 1.0e-18 * (E * E * E * E) - 1.4253 * 1.0e-12 * (E * E * E) +
                      1.2940 * 1.0e-7 * (E * E) - 5.2921 * 1.0e-3 * E + 83.3216;
        E -= E * (bias / 100);
    }
    return uint64_t(E);
}
double hll_sigma(double x) {
    if (x == 1.) return INFINITY;
    double zp, y = 1, z = x;
    do {
        x *= x;
        zp = z;
        z += x * y;
        y += y;
    } while (zp != z);
    return z;
}
double hll_tau(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zp, y = 1.0, z = 1 - x;
    do {
        x = std::sqrt(x);
        zp = z;
        y *= 0.5;
        z -= std::pow(1 - x, 2) * y;
    } while (zp != z);
    return z / 3;
}
uint64_t estimate_v5(const uint32_t *hist) {
    double m = 16384;
    double z = m * hll_tau((m - hist[51]) / m);
    for (int j = 50; j >= 1; --j) {
        z += hist[j];
        z *= 0.5;
    }
    z += m * hll_sigma(hist[0] / m);
    return uint64_t(llroundl(0.721347520444481703680 * m * m / z));
}
bool hist_exact_v3(const uint32_t *hist) {
    for (int v = 40; v < 64; v++)
        if (hist[v]) return false;
    return true;
}
// Redis-ordered sums, needed only when a register >= 40 (3.x estimator)
double dense_sum(const uint8_t *r, int *ez) {
    double E = 0;
    int z = 0;
    for (int j = 0; j < 1024; j++, r += 16) {
        for (int t = 0; t < 16; t++) z += (r[t] == 0);
        E += (g_pe[r[0]] + g_pe[r[1]]) + (g_pe[r[2]] + g_pe[r[3]]) + (g_pe[r[4]] + g_pe[r[5]]) +
             (g_pe[r[6]] + g_pe[r[7]]) + (g_pe[r[8]] + g_pe[r[9]]) + (g_pe[r[10]] + g_pe[r[11]]) +
             (g_pe[r[12]] + g_pe[r[13]]) + (g_pe[r[14]] + g_pe[r[15]]);
    }
    *ez = z;
    return E;
}
double raw_sum(const uint8_t *r, int *ez) {
    double E = 0;
    int z = 0;
    for (int j = 0; j < 2048; j++, r += 8) {
        uint64_t w;
        std::memcpy(&w, r, 8);
        if (w == 0) {
            z += 8;
            continue;
        }
        for (int t = 0; t < 8; t++) {
            if (r[t]) E += g_pe[r[t]];
            else z++;
        }
    }
    E += z;
    *ez = z;
    return E;
}

} // namespace


struct sk_ctx {
    std::mutex mu;
    int device = 0;
    int redis_major = 3;
    uint64_t max_bit_offset = 1ULL << 32;
    uint64_t max_batch = 1ULL << 22;
    hipStream_t st = nullptr;
    std::string err;

    std::unordered_map<std::string, KeyEnt> keys;
    std::unordered_map<std::string, BloomCfg> bloom; // keyed by "{name}__config"
    uint64_t bloom_seq = 0;                          // next BloomCfg::seq

    // HLL arena: slab id -> arena + id*16 KiB; free slabs are kept zeroed
    uint8_t *arena = nullptr;
    uint64_t hll_cap = 0, hll_next = 0;
    std::vector<uint32_t> hll_free;
    uint64_t hll_retired = 0;      // slabs whose generation wrapped: never handed out again (stale handles stay stale)
    uint64_t hll_epoch = 0;        // bumped whenever an HLL key is created or removed (sk_hll_epoch: cached id sets)
    std::vector<uint8_t> hll_live; // slab id -> 1 while a key owns it (caller-cached ids are checked against it)
    std::vector<uint8_t> hll_gen;  // slab id -> generation, bumped when the slab is freed (top byte of a handle)
    std::vector<uint64_t> h_e0, h_off; // host PFADD staging, kept across calls (no page faults per batch)

    // strings: host mirror of {ptr, cap}; len lives in the device directory
    std::vector<DirEnt> strs;
    std::vector<uint32_t> str_free;
    DirEnt *d_dir = nullptr;
    uint64_t dir_cap = 0;

    // in-library kernel timing (sk_prof_*): event pairs around the hot launches
    bool prof = false;
    struct ProfRec {
        int phase;
        hipEvent_t a, b;
    };
    std::vector<ProfRec> prof_pending;
    std::vector<hipEvent_t> ev_pool;
    uint32_t prof_mask = 0xffffffffu; // phases timed when prof is on (sk_prof_only)
    double prof_ms[32] = {0};
    uint64_t prof_n[32] = {0};
    hipEvent_t timers[16] = {};
    // completion tickets (sk_ticket): events on the main and read streams
    std::unordered_map<uint64_t, std::pair<hipEvent_t, hipEvent_t>> tickets;
    uint64_t next_ticket = 1;

    // cross-GPU exchange (RCCL over xGMI)
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_size = 0;
    DBuf rt_cnt;                // range-sharded RBitSet routing: per-(shard, block) counts, then their scan
    // host -> device staging of caller host buffers (stage_h2d): a ring of stage_bufs pinned buffers
    uint8_t *stage[8] = {};
    hipEvent_t stage_ev[8] = {};
    bool stage_on = false;      // SK_STAGE=1: stage pageable inputs through the ring below
    uint64_t stage_piece = 4ull << 20; // bytes per staged piece (SK_STAGE_PIECE_KB)
    uint32_t stage_bufs = 4;    // pinned buffers in the ring (SK_STAGE_BUFS, <= 8)

    bool async_dev = false;     // sk_set_async: _dev calls return without a final sync
    int pfadd_path = 1;         // 1: the partition path + line schedule (the only one since round 6)
    bool pfp_direct = true;     // partition path, one element per command: apply writes replies (SK_PFP_DIRECT)
    uint64_t sbv_min = 1u << 20; // SETBIT_VOID batches from which a dense one takes the region path (SK_SBV_MIN)
    bool sbv_part = true;       // ... through the hand-written partition (SK_SBV_PART=0: the rocPRIM radix sort)
    int read_stream = 1;        // async Bloom contains on the read stream st2 (SK_READ_STREAM=0: main stream)
    int bloom_sched = 0;        // contains kernel (SK_BLOOM_SCHED): 0 one element per thread; 1 probe queue, 4/lane; 3 split hash / probe passes
    // async PFADD: the conflict count of the last sparse batch is checked ("settled")
    // by the next call that needs the HLL arena, not by the call itself
    bool pf_pending = false;
    uint8_t *pf_changed = nullptr;
    // read stream: async Bloom contains runs beside the main stream; writers
    // on the main stream wait for ev_r, the read stream waits for ev_w when the
    // main stream may have written bit strings since it last waited (every API
    // call through ENTER may; device PFADD batches touch only the HLL arena)
    bool st_wrote_bits = true;
    hipStream_t st2 = nullptr;
    hipEvent_t ev_w = nullptr, ev_r = nullptr;
    bool rd_pending = false;
    uint32_t *h_cnt = nullptr;  // pinned, device-mapped word: conflict count written by the kernel
    uint32_t *d_h_cnt = nullptr;

    // workspace
    uint32_t *d_zero = nullptr; // device u32[4] zeros: id 0 / empty length
    DBuf keys_a, keys_b, vals_a, vals_b, sort_tmp, in_off, in_bytes, in_ids, in_cmd, out_u8, misc, partial, hist,
        uni, ptrs, hist_a, hist_b, ovf, bloom_h;
    DBuf rc_S, rc_St, rc_rec;   // Bloom contains region schedule: segment table (+ the hash's interleaved one), records
    DBuf rc_Z, rc_GT;           // ... and its zero lists: per-region lists + the (region, reply group) run table
    DBuf in_soff, in_sbytes;    // host ingress in prefix form: suffix offsets (u32) and bytes, before the rebuild
    DBuf long_h, long_which;    // PFADD: hashes of long elements (k_ms_rounds) and their element indexes + layout
    DBuf long_plane, long_flags; // their k bit planes and look-back flags
    uint64_t long_fallbacks = 0; // calls whose long elements were re-hashed per thread (look-back wait ran out)
    // device PFADD batches, pipelined (SK_PFP_PIPE, default on): batch i+1's k_pfp_hash runs on st3 while batch i's
    // k_pfp_apply runs on st; two scratch sets alternate, events order hash -> apply and apply -> reuse
    struct PfpSet {
        DBuf chunks, rep, S, big_k, big_v, ovf;
        hipEvent_t hashed = nullptr, applied = nullptr;
        bool used = false;
    } pfs[2];
    int pf_par = 0;
    bool pfp_pipe = false;      // SK_PFP_PIPE=1: the next 1 M batch hashes on a second stream while one applies (round 6 A/B: 10.4 vs 11.4 G/s without, packed arena)
    bool pf_dev_call = false;   // inside sk_pfadd_dev: inputs are caller-owned device memory, no host staging
    hipStream_t st3 = nullptr;
    // Redis HLL strings byte for byte (sk_hll_exact_strings; off by default): per slab header + sparse opcodes,
    // the apply kernel's log of register rises (records) replayed in batch order
    bool hll_exact = false;
    std::vector<HllStr> hstr;
    DBuf ev, ev_n;
    uint64_t bloom_ra_min = 1;  // add batches >= this use the region schedule (SK_BLOOM_RA_MIN, 0 = never: sort path)
    DBuf ra_S, ra_St, ra_rec, ra_flag, ra_Z, ra_GT; // Bloom add region schedule (+ its one lists and their run table)
    uint64_t bloom_rc_min = 2u << 20; // contains batches >= this use the region schedule (SK_BLOOM_RC_MIN, 0 = never)
    // PFADD line schedule (sketch-major group apply with the registers in LDS) for device batches of at least
    // pfl_min one-element commands (SK_PFL_MIN, 0 = never): scratch of one call
    uint64_t pfl_min = 4u << 20;
    uint64_t pfl_ratio = 160;   // ... and at least this many elements per sketch of the store (SK_PFL_RATIO)
    uint32_t pfl_tile = 0;      // hash blocks per run tile (SK_PFL_TILE, 0 = the kernel default)
    bool pfl_zero = true;       // replies pre-zeroed, the apply stores only the 1s (SK_PFL_ZERO)
    bool pfl_plan = true;       // heavy fine buckets dispatched first (SK_PFL_PLAN)
    DBuf pfl_chunks, pfl_S, pfl_C, pfl_rec, pfl_bk, pfl_bv, pfl_ovf, pfl_order;
    DBuf pfl_rc;                // u32[32]: reply-mix counters that pick each call's reply default (two parities)
    uint32_t pfl_par = 0;       // this call's parity
};

namespace {

int fail(sk_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
    return code;
}
#define HIPCHK(c, expr)                                                                                                \
    do {                                                                                                               \
        hipError_t e__ = (expr);                                                                                       \
        if (e__ != hipSuccess) return fail((c), SK_EDEVICE, "HIP error %s at %s:%d", hipGetErrorString(e__), __FILE__, \
                                           __LINE__);                                                                  \
    } while (0)

const char *kWrongType = "WRONGTYPE Operation against a key holding the wrong kind of value";
const char *kNotHll = "WRONGTYPE Key is not a valid HyperLogLog string value.";
const char *kRange = "ERR bit offset is not an integer or out of range";
const char *kCfgChanged = "ERR Error running script: Bloom filter config has been changed";
const char *kNotInit = "Bloom filter is not initialized!";

std::string key_of(const uint8_t *b, uint64_t len) { return std::string(reinterpret_cast<const char *>(b), len); }
std::string key_at(const uint64_t *off, const uint8_t *bytes, uint64_t i) {
    return std::string(reinterpret_cast<const char *>(bytes + off[i]), off[i + 1] - off[i]);
}

int sync(sk_ctx *c) {
    HIPCHK(c, hipStreamSynchronize(c->st));
    if (c->st2) HIPCHK(c, hipStreamSynchronize(c->st2));
    if (c->st3) HIPCHK(c, hipStreamSynchronize(c->st3));
    return SK_OK;
}

int pfadd_settle(sk_ctx *c); // defined with the PFADD core

// entry of every API call: bind the device, finish a pending async PFADD,
// and order this call after outstanding read-stream work
#define ENTER(c)                                                                                                       \
    do {                                                                                                               \
        HIPCHK(c, hipSetDevice((c)->device));                                                                          \
        (c)->st_wrote_bits = true;                                                                                     \
        if ((c)->pf_pending) {                                                                                         \
            int r__ = pfadd_settle(c);                                                                                 \
            if (r__) return r__;                                                                                       \
        }                                                                                                              \
        if ((c)->rd_pending) {                                                                                         \
            HIPCHK(c, hipStreamWaitEvent((c)->st, (c)->ev_r, 0));                                                      \
            (c)->rd_pending = false;                                                                                   \
        }                                                                                                              \
    } while (0)

// phases timed by sk_prof_* (index = SK_PROF_* in the header)
const char *kPhaseNames[] = {"pfadd_hash",  "pfadd_sort",   "pfadd_apply", "hll_hist",     "hll_union",
                             "bloom_contains", "bloom_probes", "bloom_sort", "bloom_apply", "setbit",
                             "getbit",      "bitcount",     "bitop",       "pfadd_claim", "pfadd_commit",
                             "pfp_hash",    "pfp_apply",    "pfp_reply",   "bloom_rc_hash", "bloom_rc_probe", "pfadd",
                             "pfadd_long",  "bloom_ra_hash", "bloom_ra_apply", "pfl_hash",   "pfl_part",
                             "pfl_apply",   "hll_sum",      "pfl_fill"};
constexpr int kNumPhases = sizeof(kPhaseNames) / sizeof(kPhaseNames[0]);
static_assert(kNumPhases <= 32, "prof_ms / prof_n / prof_mask hold 32 phases");

hipEvent_t ev_get(sk_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
struct Prof { // RAII: events around one launch when profiling is on
    sk_ctx *c;
    int phase;
    hipStream_t s;
    hipEvent_t a = nullptr;
    Prof(sk_ctx *c_, int ph, hipStream_t s_ = nullptr) : c(c_), phase(ph), s(s_ ? s_ : c_->st) {
        if (c->prof && (c->prof_mask >> phase & 1u)) {
            a = ev_get(c);
            (void)hipEventRecord(a, s);
        }
    }
    ~Prof() {
        if (a) {
            hipEvent_t b = ev_get(c);
            (void)hipEventRecord(b, s);
            c->prof_pending.push_back({phase, a, b});
        }
    }
};
void prof_collect(sk_ctx *c) {
    if (c->prof_pending.empty()) return;
    (void)hipStreamSynchronize(c->st);
    if (c->st2) (void)hipStreamSynchronize(c->st2);
    if (c->st3) (void)hipStreamSynchronize(c->st3);
    for (auto &r : c->prof_pending) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            c->prof_ms[r.phase] += ms;
            c->prof_n[r.phase] += 1;
        }
        c->ev_pool.push_back(r.a);
        c->ev_pool.push_back(r.b);
    }
    c->prof_pending.clear();
}

// --------------------------------------------------------------- HLL slabs
int hll_grow(sk_ctx *c, uint64_t need) {
    if (need <= c->hll_cap) return SK_OK;
    uint64_t nc = std::max<uint64_t>(need, c->hll_cap * 2);
    uint8_t *na = nullptr;
    // + 16 B: a register read takes the byte after its field (the last slab's last register included)
    if (hipMalloc(&na, nc * kSlabBytes + 16) != hipSuccess)
        return fail(c, SK_ENOMEM, "cannot allocate %llu HLL slabs", (unsigned long long)nc);
    HIPCHK(c, hipMemsetAsync(na + c->hll_cap * kSlabBytes, 0, (nc - c->hll_cap) * kSlabBytes + 16, c->st));
    if (c->arena) {
        HIPCHK(c, hipMemcpyAsync(na, c->arena, c->hll_cap * kSlabBytes, hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
        HIPCHK(c, hipFree(c->arena));
    }
    c->arena = na;
    c->hll_cap = nc;
    return SK_OK;
}

// ------------------------------------------------ Redis HLL strings, exact (sk_hll_exact_strings)




// the register rises of one PFADD launch (apply-kernel records, any order) in batch order
void hll_replay_rises(sk_ctx *c, std::vector<uint64_t> &ev) {
    std::sort(ev.begin(), ev.end(), [](uint64_t a, uint64_t b) { return ((a >> 6) & 0xfffffu) < ((b >> 6) & 0xfffffu); });
    for (uint64_t rec : ev) {
        const uint64_t slot = rec >> 26;
        const uint32_t slab = uint32_t(slot >> 14) & 0xffffffu, reg = uint32_t(slot & 16383u);
        if (slab >= c->hstr.size()) continue;
        HllStr &h = c->hstr[slab];
        h.hdr[15] |= 0x80; // PFADD updated: HLL_INVALIDATE_CACHE
        if (!h.sparse) continue;
        int r = hll_sparse_set(h, reg, uint8_t(rec & 63u));
        if (r == 2 || r < 0) hll_str_densify(h);
    }
}

// single-key PFCOUNT (pfcountCommand): a valid cached cardinality answers; a stale one is replaced by the count
void hll_card_cache(sk_ctx *c, uint32_t slab, int64_t *count) {
    if (!c->hll_exact || slab >= c->hstr.size()) return;
    HllStr &h = c->hstr[slab];
    if (!(h.hdr[15] & 0x80)) {
        uint64_t v = 0;
        for (int i = 7; i >= 0; i--) v = (v << 8) | h.hdr[8 + i];
        *count = int64_t(v);
        return;
    }
    const uint64_t v = uint64_t(*count);
    for (int i = 0; i < 8; i++) h.hdr[8 + i] = uint8_t(v >> (8 * i));
}

// PFMERGE destination (pfmergeCommand): made dense, cached cardinality stale
void hll_str_merged(sk_ctx *c, uint32_t slab) {
    if (!c->hll_exact || slab >= c->hstr.size()) return;
    hll_str_densify(c->hstr[slab]);
    c->hstr[slab].hdr[15] |= 0x80;
}

// H2D of a caller's host range, asynchronous on c->st.  With SK_STAGE=1, large pageable ranges go through a ring of
// stage_bufs pinned buffers of stage_piece bytes (SK_STAGE_BUFS, SK_STAGE_PIECE_KB): host threads copy piece p into
// buffer p % stage_bufs while the device copies the pieces before it at the link's rate.  A buffer is refilled only
// after the event of its previous copy completed.  Off by default: measured, the runtime's own staging of a pageable
// hipMemcpyAsync was as fast or faster (host ingress).  Pinned caller memory (a buffer the JNI side
// allocated with sk_host_alloc) is always copied directly.
int stage_h2d(sk_ctx *c, void *dst, const void *src, uint64_t bytes) {
    if (!bytes) return SK_OK;
    hipPointerAttribute_t at;
    const bool pinned = hipPointerGetAttributes(&at, src) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError(); // pageable memory reports an error here
    if (!c->stage_on || pinned || bytes < 2 * c->stage_piece) {
        HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->st));
        return SK_OK;
    }
    const uint32_t nb = c->stage_bufs;
    for (uint32_t k = 0; k < nb; k++)
        if (!c->stage[k]) {
            HIPCHK(c, hipHostMalloc((void **)&c->stage[k], c->stage_piece, hipHostMallocDefault));
            HIPCHK(c, hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming));
            HIPCHK(c, hipEventRecord(c->stage_ev[k], c->st));
        }
    // a ring of nb pinned buffers: host threads fill piece p into buffer p % nb while the DMA engine copies the
    // pieces before it; a buffer is refilled once the event of its previous copy completed
    const uint8_t *s8 = static_cast<const uint8_t *>(src);
    uint8_t *d8 = static_cast<uint8_t *>(dst);
    for (uint64_t o = 0, p = 0; o < bytes; o += c->stage_piece, p++) {
        const uint32_t k = uint32_t(p % nb);
        const uint64_t len = std::min(c->stage_piece, bytes - o);
        HIPCHK(c, hipEventSynchronize(c->stage_ev[k]));
        host_for(len, 256u << 10, [&](uint64_t a, uint64_t b) { std::memcpy(c->stage[k] + a, s8 + o + a, b - a); });
        HIPCHK(c, hipMemcpyAsync(d8 + o, c->stage[k], len, hipMemcpyHostToDevice, c->st));
        HIPCHK(c, hipEventRecord(c->stage_ev[k], c->st));
    }
    return SK_OK;
}

int hll_alloc(sk_ctx *c, uint32_t *id) {
    if (!c->hll_free.empty()) {
        *id = c->hll_free.back();
        c->hll_free.pop_back();
    } else {
        if (c->hll_next >= (uint64_t(1) << 24))
            return fail(c, SK_ENOMEM, "too many HLL keys: %llu slabs (2^24 per context)", (unsigned long long)c->hll_next);
        int r = hll_grow(c, c->hll_next + 1);
        if (r) return r;
        *id = uint32_t(c->hll_next++);
    }
    if (c->hll_live.size() <= *id) {
        size_t n = std::max<size_t>(*id + 1, c->hll_live.size() * 2);
        c->hll_live.resize(n, 0);
        c->hll_gen.resize(n, 0);
    }
    c->hll_live[*id] = 1;
    c->hll_epoch++;
    if (c->hll_exact) {
        if (c->hstr.size() <= *id) c->hstr.resize(std::max<size_t>(*id + 1, c->hstr.size() * 2));
        hll_str_init(c->hstr[*id]);
    }
    return SK_OK;
}
// Caller-cached handles (sk_hll_resolve -> sk_pfadd_ids / sk_pfcount_ids) = slab | generation << 24: usable only
// while the key that was resolved still owns the slab (a DEL / SET / BITOP / flushall frees it and bumps the
// generation, so a handle cached across that -- even with the slab handed to another key -- is refused).
constexpr uint32_t kSlabMask = 0xffffffu;
uint32_t hll_handle(const sk_ctx *c, uint32_t id) { return id | (uint32_t(c->hll_gen[id]) << 24); }
bool hll_handle_live(const sk_ctx *c, uint32_t h) {
    uint32_t id = h & kSlabMask;
    return id < c->hll_live.size() && c->hll_live[id] && c->hll_gen[id] == (h >> 24);
}
// index of the first handle of ids[0..n) that is not live, or n: on host threads for large batches (the check of
// caller-cached handles must not cost more than the batch's H2D)
uint64_t first_dead_handle(const sk_ctx *c, uint64_t n, const uint32_t *ids) {
    std::atomic<uint64_t> bad{n};
    host_for(n, 1u << 16, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; i++)
            if (!hll_handle_live(c, ids[i])) {
                uint64_t cur = bad.load();
                while (i < cur && !bad.compare_exchange_weak(cur, i)) {
                }
                return;
            }
    });
    return bad.load();
}

int str_len(sk_ctx *c, uint32_t id, uint64_t *len);
int str_free(sk_ctx *c, uint32_t id);


// A string key holding a Redis HLL (SET / restore of a redis-server value)
// becomes an HLL key the first time an HLL command touches it, as redis-server
// accepts any string with a valid HLL encoding.  Its cached cardinality is
// not kept: PFCOUNT recomputes it.
int hll_adopt_string(sk_ctx *c, const std::string &k, KeyEnt &e, uint32_t *id) {
    uint64_t l;
    int r = str_len(c, e.id, &l);
    if (r) return r;
    if (l < 16 || l > 16 + 2 * 16384) return fail(c, SK_EWRONGTYPE, "%s", kNotHll);
    std::vector<uint8_t> s(l), regs(kHllBytes, 0);
    HIPCHK(c, hipMemcpyAsync(s.data(), c->strs[e.id].ptr, l, hipMemcpyDeviceToHost, c->st));
    if ((r = sync(c))) return r;
    r = hll_decode(s.data(), l, regs.data());
    if (r == SK_EWRONGTYPE) return fail(c, r, "%s", kNotHll);
    if (r == SK_ECORRUPT) return fail(c, r, "INVALIDOBJ Corrupted HLL object detected");
    uint32_t hid;
    if ((r = hll_alloc(c, &hid))) return r;
    if (c->hll_exact) { // the string as redis-server would keep using it: its header, its sparse opcodes
        HllStr &h = c->hstr[hid];
        std::memcpy(h.hdr, s.data(), 16);
        h.sparse = s[4] == 1;
        if (h.sparse) h.ops.assign(s.begin() + 16, s.end());
        else std::vector<uint8_t>().swap(h.ops);
    }
    std::vector<uint8_t> body(kSlabBytes);
    hll_body_pack(regs.data(), body.data());
    HIPCHK(c, hipMemcpyAsync(c->arena + uint64_t(hid) * kSlabBytes, body.data(), kSlabBytes, hipMemcpyHostToDevice,
                             c->st));
    if ((r = sync(c))) return r;
    if ((r = str_free(c, e.id))) return r;
    e = KeyEnt{SK_TYPE_HLL, hid};
    *id = hid;
    (void)k;
    return SK_OK;
}

// lookup or create an HLL key (PFADD / PFMERGE create)
int hll_get(sk_ctx *c, const std::string &k, bool create, uint32_t *id, bool *created) {
    if (created) *created = false;
    auto it = c->keys.find(k);
    if (it != c->keys.end()) {
        if (it->second.type == SK_TYPE_STRING) return hll_adopt_string(c, k, it->second, id);
        if (it->second.type != SK_TYPE_HLL) return fail(c, SK_EWRONGTYPE, "%s", kNotHll);
        *id = it->second.id;
        return SK_OK;
    }
    if (!create) {
        *id = kNoId;
        return SK_OK;
    }
    int r = hll_alloc(c, id);
    if (r) return r;
    c->keys[k] = KeyEnt{SK_TYPE_HLL, *id};
    if (created) *created = true;
    return SK_OK;
}

// -------------------------------------------------------------- strings
int dir_write(sk_ctx *c, uint32_t id, const DirEnt &e) {
    HIPCHK(c, hipMemcpyAsync(c->d_dir + id, &e, sizeof(DirEnt), hipMemcpyHostToDevice, c->st));
    return SK_OK;
}
int str_len(sk_ctx *c, uint32_t id, uint64_t *len) {
    HIPCHK(c, hipMemcpyAsync(len, &c->d_dir[id].len, sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    return sync(c);
}
int str_set_len(sk_ctx *c, uint32_t id, uint64_t len) {
    HIPCHK(c, hipMemcpyAsync(&c->d_dir[id].len, &len, sizeof(uint64_t), hipMemcpyHostToDevice, c->st));
    return sync(c); // len is a stack variable
}

int str_alloc(sk_ctx *c, uint64_t cap, uint32_t *id) {
    cap = round16(std::max<uint64_t>(cap, 16));
    uint8_t *p = nullptr;
    if (hipMalloc(&p, cap) != hipSuccess)
        return fail(c, SK_ENOMEM, "cannot allocate %llu-byte string", (unsigned long long)cap);
    HIPCHK(c, hipMemsetAsync(p, 0, cap, c->st));
    uint32_t nid;
    if (!c->str_free.empty()) {
        nid = c->str_free.back();
        c->str_free.pop_back();
    } else {
        nid = uint32_t(c->strs.size());
        c->strs.push_back(DirEnt{nullptr, 0, 0});
    }
    if (c->strs.size() > c->dir_cap) {
        uint64_t nc = std::max<uint64_t>(64, c->dir_cap * 2);
        DirEnt *nd = nullptr;
        HIPCHK(c, hipMalloc(&nd, nc * sizeof(DirEnt)));
        if (c->d_dir) {
            HIPCHK(c, hipMemcpyAsync(nd, c->d_dir, c->dir_cap * sizeof(DirEnt), hipMemcpyDeviceToDevice, c->st));
            HIPCHK(c, hipStreamSynchronize(c->st));
            HIPCHK(c, hipFree(c->d_dir));
        }
        c->d_dir = nd;
        c->dir_cap = nc;
    }
    c->strs[nid] = DirEnt{p, 0, cap};
    *id = nid;
    int r = dir_write(c, nid, c->strs[nid]);
    if (r) return r;
    return sync(c);
}

int str_free(sk_ctx *c, uint32_t id) {
    HIPCHK(c, hipStreamSynchronize(c->st));
    if (c->strs[id].ptr) HIPCHK(c, hipFree(c->strs[id].ptr));
    c->strs[id] = DirEnt{nullptr, 0, 0};
    c->str_free.push_back(id);
    return dir_write(c, id, c->strs[id]);
}

// grow capacity to >= need bytes (new bytes zero, content kept)
int str_reserve(sk_ctx *c, uint32_t id, uint64_t need) {
    DirEnt &e = c->strs[id];
    if (need <= e.cap) return SK_OK;
    uint64_t nc = round16(std::max(need, e.cap * 2));
    uint8_t *p = nullptr;
    if (hipMalloc(&p, nc) != hipSuccess)
        return fail(c, SK_ENOMEM, "cannot allocate %llu-byte string", (unsigned long long)nc);
    HIPCHK(c, hipMemsetAsync(p + e.cap, 0, nc - e.cap, c->st));
    HIPCHK(c, hipMemcpyAsync(p, e.ptr, e.cap, hipMemcpyDeviceToDevice, c->st));
    uint64_t len;
    int r = str_len(c, id, &len);
    if (r) return r;
    HIPCHK(c, hipFree(e.ptr));
    e.ptr = p;
    e.cap = nc;
    DirEnt w{p, len, nc};
    r = dir_write(c, id, w);
    if (r) return r;
    return sync(c);
}

// lookup or create a plain string key (SETBIT / SET / BITOP dest)
int str_get(sk_ctx *c, const std::string &k, bool create, uint64_t init_cap, uint32_t *id) {
    auto it = c->keys.find(k);
    if (it != c->keys.end()) {
        if (it->second.type != SK_TYPE_STRING) return fail(c, SK_EWRONGTYPE, "%s", kWrongType);
        *id = it->second.id;
        return SK_OK;
    }
    if (!create) {
        *id = kNoId;
        return SK_OK;
    }
    int r = str_alloc(c, init_cap, id);
    if (r) return r;
    c->keys[k] = KeyEnt{SK_TYPE_STRING, *id};
    return SK_OK;
}

int del_key(sk_ctx *c, const std::string &k, bool *removed) {
    *removed = false;
    auto b = c->bloom.find(k);
    if (b != c->bloom.end()) {
        c->bloom.erase(b);
        *removed = true;
        return SK_OK;
    }
    auto it = c->keys.find(k);
    if (it == c->keys.end()) return SK_OK;
    KeyEnt e = it->second;
    c->keys.erase(it);
    *removed = true;
    if (e.type == SK_TYPE_HLL) {
        HIPCHK(c, hipMemsetAsync(c->arena + uint64_t(e.id) * kSlabBytes, 0, kSlabBytes, c->st));
        c->hll_live[e.id] = 0;
        c->hll_epoch++;
        c->hll_gen[e.id] = uint8_t(c->hll_gen[e.id] + 1);
        // a generation that wrapped would make a handle cached 256 frees ago live again: retire the slab instead
        if (c->hll_gen[e.id] == 0) c->hll_retired++;
        else c->hll_free.push_back(e.id);
        return SK_OK;
    }
    return str_free(c, e.id);
}

// ------------------------------------------------------------ PFADD core
// Device batch: n elements with per-element slab id and command index.  Two schedules, same replies and registers:
// the partition path (k_pfp_hash / k_pfp_apply, <= 1 M elements per launch, any density) and, for a large group of
// one-element commands, the line schedule (k_pfl_*).  (Rounds 1-5 also kept a claim / commit path on the registers'
// spare bits and a radix-sorted path; the packed 6-bit arena has no spare bits, and both were retired in round 6.)
int pfadd_settle(sk_ctx *c) { // nothing is left pending by the current paths
    c->pf_pending = false;
    return SK_OK;
}

// partition path (sk_kernels.hip "PFADD, partition path"); n <= 2^20 per launch.
// Exact for every input on the device (oversized buckets: k_pfp_big), so the
// host never waits on a batch.
// pipelined form of the partition path for device-resident inputs: the hash of this batch goes to st3 (it reads
// only the caller's inputs and its own scratch set), the apply stays on st in batch order (replies and registers
// depend on the previous batch's registers, so applies never reorder)
int pfadd_partition_pipe(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint64_t *d_off, const uint8_t *d_bytes,
                         uint8_t *d_changed) {
    uint64_t nb = sk::pfp_blocks(n), cap = nb * sk::pfp_epb();
    sk_ctx::PfpSet &ps = c->pfs[c->pf_par];
    c->pf_par ^= 1;
    if (!ps.hashed) {
        HIPCHK(c, hipEventCreateWithFlags(&ps.hashed, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&ps.applied, hipEventDisableTiming));
    }
    if (ps.used) HIPCHK(c, hipStreamWaitEvent(c->st3, ps.applied, 0)); // the set's previous apply is done
    HIPCHK(c, ps.chunks.ensure(cap * 8));
    HIPCHK(c, ps.rep.ensure(cap + 32));
    HIPCHK(c, ps.S.ensure((uint64_t(sk::pfp_buckets()) + 1) * nb * 4));
    HIPCHK(c, ps.big_k.ensure(2 * n * 8));
    HIPCHK(c, ps.big_v.ensure(2 * n * 4));
    HIPCHK(c, ps.ovf.ensure(64));
    { Prof p_(c, 15, c->st3);
    HIPCHK(c, sk::launch_pfp_hash(c->st3, n, d_ids, d_off, d_bytes, c->redis_major >= 5, ps.chunks.as<uint64_t>(),
                                  ps.S.as<uint32_t>(), nullptr, ps.ovf.as<uint32_t>(), nullptr)); }
    HIPCHK(c, hipEventRecord(ps.hashed, c->st3));
    HIPCHK(c, hipStreamWaitEvent(c->st, ps.hashed, 0));
    { Prof p_(c, 16);
    HIPCHK(c, sk::launch_pfp_apply(c->st, n, ps.chunks.as<uint64_t>(), ps.S.as<uint32_t>(), c->arena,
                                   ps.rep.as<uint8_t>(), ps.ovf.as<uint32_t>(), ps.big_k.as<uint64_t>(),
                                   ps.big_v.as<uint32_t>(), d_changed)); }
    HIPCHK(c, hipEventRecord(ps.applied, c->st));
    ps.used = true;
    return SK_OK;
}

int pfadd_partition(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint64_t *d_off, const uint8_t *d_bytes,
                    const uint32_t *d_cmd, uint8_t *d_changed, const uint64_t *d_pre = nullptr) {
    if (n > (1ull << 20) || c->hll_next >= (1ull << 24)) return fail(c, SK_EINVAL, "PFADD partition batch too large");
    if (c->pf_dev_call && c->pfp_pipe && c->pfp_direct && d_cmd == nullptr && d_pre == nullptr && c->st3 &&
        !c->hll_exact)
        return pfadd_partition_pipe(c, n, d_ids, d_off, d_bytes, d_changed);
    uint64_t *ev = nullptr; // exact HLL strings: the apply kernel logs every register rise
    uint32_t *ev_n = nullptr;
    if (c->hll_exact) {
        HIPCHK(c, c->ev.ensure(n * 8));
        HIPCHK(c, c->ev_n.ensure(16));
        HIPCHK(c, hipMemsetAsync(c->ev_n.p, 0, 4, c->st));
        ev = c->ev.as<uint64_t>();
        ev_n = c->ev_n.as<uint32_t>();
    }
    uint64_t nb = sk::pfp_blocks(n), cap = nb * sk::pfp_epb();
    HIPCHK(c, c->keys_a.ensure(cap * 8));                                // block chunks of records
    HIPCHK(c, c->keys_b.ensure(cap + 2 * n + 32));                       // replies in chunk order + element slots
    HIPCHK(c, c->hist_a.ensure((uint64_t(sk::pfp_buckets()) + 1) * nb * 4)); // bucket starts per block
    HIPCHK(c, c->vals_a.ensure(2 * n * 8)); // oversized-bucket tables: 2 entries per record
    HIPCHK(c, c->vals_b.ensure(2 * n * 4));
    HIPCHK(c, c->ovf.ensure(64));
    uint64_t *chunks = c->keys_a.as<uint64_t>();
    uint8_t *rep = c->keys_b.as<uint8_t>();
    uint16_t *pos = reinterpret_cast<uint16_t *>(rep + ((cap + 15) & ~uint64_t(15)));
    uint32_t *S = c->hist_a.as<uint32_t>(), *big_alloc = c->ovf.as<uint32_t>();
    // one element per command: k_pfp_apply stores each reply at its batch position (a 1 MB reply array stays
    // in L2, so the scattered byte stores cost no HBM requests) and the order-restoring launch is skipped
    const bool direct = d_cmd == nullptr && c->pfp_direct;
    { Prof p_(c, 15);
    HIPCHK(c, sk::launch_pfp_hash(c->st, n, d_ids, d_off, d_bytes, c->redis_major >= 5, chunks, S,
                                  direct ? nullptr : pos, big_alloc, d_pre)); }
    { Prof p_(c, 16);
    HIPCHK(c, sk::launch_pfp_apply(c->st, n, chunks, S, c->arena, rep, big_alloc, c->vals_a.as<uint64_t>(),
                                   c->vals_b.as<uint32_t>(), direct ? d_changed : nullptr, ev, ev_n)); }
    if (!direct) {
        Prof p_(c, 17);
        HIPCHK(c, sk::launch_pfp_reply(c->st, n, rep, pos, d_cmd, d_changed));
    }
    if (ev) {
        uint32_t ne = 0;
        HIPCHK(c, hipMemcpyAsync(&ne, ev_n, 4, hipMemcpyDeviceToHost, c->st));
        int r = sync(c);
        if (r) return r;
        std::vector<uint64_t> h(ne);
        if (ne) HIPCHK(c, hipMemcpyAsync(h.data(), ev, uint64_t(ne) * 8, hipMemcpyDeviceToHost, c->st));
        if ((r = sync(c))) return r;
        hll_replay_rises(c, h);
    }
    return SK_OK;
}

// line schedule (sk_kernels.hip "PFADD, line schedule"): one element per command, n <= 2^26, every slab id
// below hll_next <= sk::pfl_max_slabs().  Five launches on st, no host wait, exact replies for every input.
bool pfadd_lines_ok(sk_ctx *c, uint64_t n) {
    // worth it once a call puts enough elements on each sketch: fine buckets hold <= 128 sketches, and a bucket of a
    // few dozen records costs the apply a workgroup for little work (4 M over 100 k tenants: 4.2 G/s against 9.2
    // for the partition path; 16 M: 13.5 against 9.0)
    return c->pfl_min && n >= c->pfl_min && n >= c->pfl_ratio * c->hll_next && c->pfadd_path == 1 &&
           !c->hll_exact && c->hll_next > 0 && c->hll_next <= sk::pfl_max_slabs();
}
int pfadd_lines(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint64_t *d_off, const uint8_t *d_bytes,
                uint8_t *d_changed) {
    if (n > (1ull << 26)) return fail(c, SK_EINVAL, "PFADD line batch too large");
    const uint32_t nslab = uint32_t(c->hll_next);
    const sk::PflDims d = sk::pfl_dims(n, nslab, c->pfl_tile);
    if (!sk::pfl_dims_ok(d))
        return fail(c, SK_EINVAL, "PFADD line schedule: tile of %u hash blocks out of range (SK_PFL_TILE)", d.tb);
    HIPCHK(c, c->pfl_chunks.ensure(d.chunk_bytes));
    HIPCHK(c, c->pfl_S.ensure(d.S_bytes));
    HIPCHK(c, c->pfl_C.ensure(d.c_words * 4));
    HIPCHK(c, c->pfl_rec.ensure(d.chunk_bytes)); // records: u64 or 6-B planes per hash-block slot (SK_PFL_R6)
    HIPCHK(c, c->pfl_bk.ensure(2 * n * 8));
    HIPCHK(c, c->pfl_bv.ensure(2 * n * 4));
    HIPCHK(c, c->pfl_ovf.ensure(64));
    HIPCHK(c, c->pfl_order.ensure(d.nf * 4));
    if (!c->pfl_rc.p) { // first call: no reply mix yet (default 0)
        HIPCHK(c, c->pfl_rc.ensure(32 * 4));
        HIPCHK(c, hipMemsetAsync(c->pfl_rc.p, 0, 32 * 4, c->st));
    }
    { Prof p_(c, 24);
    HIPCHK(c, sk::launch_pfl_hash(c->st, n, d_ids, d_off, d_bytes, c->redis_major >= 5, c->pfl_chunks.as<uint64_t>(),
                                  c->pfl_S.as<uint32_t>(), c->pfl_ovf.as<uint32_t>())); }
    // replies: pre-filled with the call's default (the previous call's majority reply) by one streaming kernel, then
    // the apply stores only the other replies, instead of one scattered byte per element (SK_PFL_ZERO=0: every
    // reply stored by the apply).  The fill runs before the region pass, which stores 0 for the records it drops
    // (slab id >= nslab: no register, reply 0), so the default never overwrites those.
    const uint32_t par = c->pfl_par;
    c->pfl_par ^= 1;
    { Prof p_(c, 28);
    if (c->pfl_zero) HIPCHK(c, sk::launch_pfl_fill(c->st, d_changed, n, c->pfl_rc.as<uint32_t>(), par)); }
    { Prof p_(c, 25);
    HIPCHK(c, sk::launch_pfl_part(c->st, d, c->pfl_chunks.as<uint64_t>(), c->pfl_S.as<uint32_t>(),
                                  c->pfl_C.as<uint32_t>(), c->pfl_rec.as<uint64_t>(), d_changed)); }
    { Prof p_(c, 26);
    HIPCHK(c, sk::launch_pfl_apply(c->st, d, c->pfl_rec.as<uint64_t>(), c->pfl_C.as<uint32_t>(), nslab, c->arena,
                                   d_changed, c->pfl_ovf.as<uint32_t>(), c->pfl_bk.as<uint64_t>(),
                                   c->pfl_bv.as<uint32_t>(), c->pfl_zero ? 32 : 0,
                                   c->pfl_plan ? c->pfl_order.as<uint32_t>() : nullptr, c->pfl_rc.as<uint32_t>(),
                                   par)); }
    if (getenv("SK_PFL_DEBUG")) { // dev: table entries the oversized runs took (2 per record of a min-seq table run)
        uint32_t big = 0;
        HIPCHK(c, hipMemcpyAsync(&big, c->pfl_ovf.p, 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));
        fprintf(stderr, "[pfl] n=%llu sh=%u nsub=%u ntile=%u tb=%u rcap=%u big-table records=%u\n",
                (unsigned long long)n, d.sh, d.nsub, d.ntile, d.tb, d.rcap, big / 2);
    }
    return SK_OK;
}

int pfadd_device(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint64_t *d_off, const uint8_t *d_bytes,
                 const uint32_t *d_cmd, uint64_t n_cmds, uint8_t *d_changed, uint64_t touched_keys,
                 const uint64_t *d_pre = nullptr) {
    if (!n) return SK_OK;
    if (d_cmd == nullptr && d_pre == nullptr && pfadd_lines_ok(c, n)) { // large one-element batch: line schedule
        for (uint64_t s = 0; s < n; s += (1ull << 26)) {
            int r = pfadd_lines(c, std::min<uint64_t>(1ull << 26, n - s), d_ids + s, d_off + s, d_bytes, d_changed + s);
            if (r) return r;
        }
        return SK_OK;
    }
    if (c->pfadd_path == 1) { // partition path, 1M elements per launch
        for (uint64_t s = 0; s < n; s += (1ull << 20)) {
            if (c->pf_pending) {
                int r = pfadd_settle(c);
                if (r) return r;
            }
            uint64_t m = std::min<uint64_t>(1ull << 20, n - s);
            const uint64_t *pre = d_pre ? d_pre + s : nullptr;
            // element offsets stay absolute; the command index of element s+j is d_cmd[s+j] (or s+j)
            if (d_cmd == nullptr && s > 0) {
                int r = pfadd_partition(c, m, d_ids + s, d_off + s, d_bytes, nullptr, d_changed + s, pre);
                if (r) return r;
            } else if (d_cmd == nullptr) {
                int r = pfadd_partition(c, m, d_ids, d_off, d_bytes, nullptr, d_changed, pre);
                if (r) return r;
            } else {
                int r = pfadd_partition(c, m, d_ids + s, d_off + s, d_bytes, d_cmd + s, d_changed, pre);
                if (r) return r;
            }
        }
        return SK_OK;
    }
    return fail(c, SK_EINVAL, "PFADD path %d is retired (the partition path is 1)", c->pfadd_path);
}

// base: the packed arena (slab ids), or a u8 register array (d_ids = d_zero)
int hll_histograms(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint8_t *base, std::vector<uint32_t> &h) {
    HIPCHK(c, c->hist.ensure(n * 64 * 4));
    { Prof p_(c, 3);
    HIPCHK(c, sk::launch_hll_hist(c->st, n, d_ids, base, c->hist.as<uint32_t>(), base == c->arena ? 1 : 0)); }
    h.resize(n * 64);
    HIPCHK(c, hipMemcpyAsync(h.data(), c->hist.p, n * 64 * 4, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

// register max of slabs `ids` into d_out: u8 registers, or a packed slab of the arena (out_slab)
int union_into(sk_ctx *c, const std::vector<uint32_t> &ids, uint8_t *d_out, int include_out, int out_slab) {
    HIPCHK(c, c->in_ids.ensure(std::max<size_t>(ids.size(), 1) * 4));
    if (!ids.empty())
        HIPCHK(c, hipMemcpyAsync(c->in_ids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, c->st));
    const uint64_t max_groups = 4096;
    HIPCHK(c, c->partial.ensure((max_groups + max_groups / 64 + 2) * kHllBytes));
    HIPCHK(c, sk::launch_hll_union(c->st, ids.size(), c->in_ids.as<uint32_t>(), c->arena, c->partial.as<uint8_t>(),
                                   max_groups, d_out, include_out, 1, out_slab));
    return sync(c); // ids is a host vector
}

// d_regs: u8 registers on the device, or (packed) a slab of the arena
uint64_t estimate_host(sk_ctx *c, const uint32_t *hist, const uint8_t *d_regs, bool raw_order, int *rc,
                       bool packed = false) {
    *rc = SK_OK;
    if (c->redis_major >= 5) return estimate_v5(hist);
    if (hist_exact_v3(hist)) {
        double E = 0;
        for (int v = 0; v < 64; v++) E += double(hist[v]) * g_pe[v]; // every partial sum exact
        return estimate_v3(E, int(hist[0]));
    }
    // a register >= 40: the summation order matters -> redo it in Redis order
    std::vector<uint8_t> regs(kHllBytes), body(packed ? kSlabBytes : 0);
    if (hipMemcpy(packed ? body.data() : regs.data(), d_regs, packed ? kSlabBytes : kHllBytes, hipMemcpyDeviceToHost) !=
        hipSuccess) {
        *rc = fail(c, SK_EDEVICE, "register readback failed");
        return 0;
    }
    if (packed) hll_body_unpack(body.data(), regs.data());
    int ez;
    double E = raw_order ? raw_sum(regs.data(), &ez) : dense_sum(regs.data(), &ez);
    return estimate_v3(E, ez);
}

// ------------------------------------------------------------- bit strings
int check_offsets(sk_ctx *c, uint64_t n, const uint64_t *offs, std::vector<uint8_t> &ok) {
    ok.assign(n, 1);
    int r = SK_OK;
    for (uint64_t i = 0; i < n; i++)
        if (offs[i] >= c->max_bit_offset) {
            ok[i] = 0;
            r = fail(c, SK_ERANGE, "%s", kRange);
        }
    return r;
}

int bloom_cfg(sk_ctx *c, const std::string &name, BloomCfg **out) {
    auto it = c->bloom.find("{" + name + "}__config");
    if (it == c->bloom.end()) return fail(c, SK_ENOTINIT, "%s", kNotInit);
    *out = &it->second;
    return SK_OK;
}

uint64_t magic_for(uint64_t d) { return ~0ull / d; }

} // namespace

// =================================================================== C ABI
extern "C" {

const char *sk_strerror(int s) {
    switch (s) {
    case SK_OK: return "OK";
    case SK_EWRONGTYPE: return kWrongType;
    case SK_ERANGE: return kRange;
    case SK_ECONFIG: return kCfgChanged;
    case SK_ENOTINIT: return kNotInit;
    case SK_EDEVICE: return "device error";
    case SK_EINVAL: return "invalid argument";
    case SK_ENOMEM: return "out of memory";
    case SK_ESYNTAX: return "ERR BITOP NOT must be called with a single source key.";
    case SK_ETOOBIG: return "Bloom filter can't be greater than 4294967294";
    case SK_ECORRUPT: return "INVALIDOBJ Corrupted HLL object detected";
    case SK_ESTALE: return "stale HLL slab id: resolve the key again";
    case SK_EBUSYKEY: return "BUSYKEY Target key name already exists.";
    case SK_EPAYLOAD: return "ERR DUMP payload version or checksum are wrong";
    default: return "unknown";
    }
}

int sk_open(const sk_config *cfg, sk_ctx **out) {
    if (!out) return SK_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return SK_EDEVICE;
    sk_ctx *c = new sk_ctx();
    if (cfg) {
        c->device = cfg->device;
        c->redis_major = cfg->redis_major ? cfg->redis_major : 3;
        if (cfg->max_bit_offset) c->max_bit_offset = cfg->max_bit_offset;
        if (cfg->max_batch) c->max_batch = cfg->max_batch;
    }
    // stream priorities (SK_STREAM_PRIO): 0 both normal, 1 main (write) stream high, 2 read stream high
    int prio_mode = 0, lo = 0, hi = 0;
    if (const char *e = getenv("SK_STREAM_PRIO")) prio_mode = atoi(e);
    if (c->device < 0 || c->device >= ndev || hipSetDevice(c->device) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, prio_mode == 1 ? hi : lo) != hipSuccess ||
        hipStreamCreateWithPriority(&c->st2, hipStreamNonBlocking, prio_mode == 2 ? hi : lo) != hipSuccess ||
        hipStreamCreateWithPriority(&c->st3, hipStreamNonBlocking, lo) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_w, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_r, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return SK_EDEVICE;
    }
    if (const char *e = getenv("SK_BLOOM_SCHED")) c->bloom_sched = atoi(e);
    if (const char *e = getenv("SK_READ_STREAM")) c->read_stream = atoi(e);
    if (const char *e = getenv("SK_PFADD_PATH")) c->pfadd_path = atoi(e);
    if (const char *e = getenv("SK_PFP_DIRECT")) c->pfp_direct = atoi(e) != 0;
    if (const char *e = getenv("SK_SBV_MIN")) c->sbv_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("SK_SBV_PART")) c->sbv_part = atoi(e) != 0;
    if (const char *e = getenv("SK_BLOOM_RC_MIN")) c->bloom_rc_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("SK_BLOOM_RA_MIN")) c->bloom_ra_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("SK_HLL_EXACT_STRINGS")) c->hll_exact = atoi(e) != 0;
    if (c->hll_exact) c->pfadd_path = 1;
    if (const char *e = getenv("SK_PFP_PIPE")) c->pfp_pipe = atoi(e) != 0;
    if (const char *e = getenv("SK_PFL_MIN")) c->pfl_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("SK_PFL_RATIO")) c->pfl_ratio = strtoull(e, nullptr, 10);
    if (const char *e = getenv("SK_PFL_TILE")) c->pfl_tile = uint32_t(strtoul(e, nullptr, 10));
    if (const char *e = getenv("SK_PFL_ZERO")) c->pfl_zero = atoi(e) != 0;
    if (const char *e = getenv("SK_PFL_PLAN")) c->pfl_plan = atoi(e) != 0;
    if (const char *e = getenv("SK_STAGE")) c->stage_on = atoi(e) != 0;
    if (const char *e = getenv("SK_STAGE_PIECE_KB")) c->stage_piece = std::max<uint64_t>(64, strtoull(e, nullptr, 10)) << 10;
    if (const char *e = getenv("SK_STAGE_BUFS")) c->stage_bufs = uint32_t(std::min(8, std::max(2, atoi(e))));
    uint64_t cap = (cfg && cfg->hll_capacity) ? cfg->hll_capacity : 1024;
    if (hll_grow(c, cap) != SK_OK || c->misc.ensure(4096) != hipSuccess ||
        hipMalloc(&c->d_zero, 16) != hipSuccess || hipMemsetAsync(c->d_zero, 0, 16, c->st) != hipSuccess ||
        hipHostMalloc((void **)&c->h_cnt, 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->d_h_cnt, c->h_cnt, 0) != hipSuccess ||
        hipMemsetAsync(c->misc.p, 0, 4096, c->st) != hipSuccess || hipStreamSynchronize(c->st) != hipSuccess) {
        sk_close(c);
        return SK_EDEVICE;
    }
    *out = c;
    return SK_OK;
}

int sk_close(sk_ctx *c) {
    if (!c) return SK_OK;
    (void)hipSetDevice(c->device);
    if (c->pf_pending) (void)pfadd_settle(c);
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->st2) (void)hipStreamSynchronize(c->st2);
    if (c->st3) (void)hipStreamSynchronize(c->st3);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    prof_collect(c);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    for (auto &t : c->tickets) (void)hipEventDestroy(t.second.first), (void)hipEventDestroy(t.second.second);
    for (hipEvent_t e : c->timers)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : c->strs)
        if (e.ptr) (void)hipFree(e.ptr);
    if (c->arena) (void)hipFree(c->arena);
    if (c->d_dir) (void)hipFree(c->d_dir);
    if (c->d_zero) (void)hipFree(c->d_zero);
    if (c->h_cnt) (void)hipHostFree(c->h_cnt);
    for (int k = 0; k < 8; k++) {
        if (c->stage[k]) (void)hipHostFree(c->stage[k]);
        if (c->stage_ev[k]) (void)hipEventDestroy(c->stage_ev[k]);
    }
    for (DBuf *b : {&c->keys_a, &c->keys_b, &c->vals_a, &c->vals_b, &c->sort_tmp, &c->in_off, &c->in_bytes,
                    &c->in_ids, &c->in_cmd, &c->out_u8, &c->misc, &c->partial, &c->hist, &c->uni, &c->ptrs,
                    &c->hist_a, &c->hist_b, &c->ovf, &c->bloom_h, &c->rc_S, &c->rc_St, &c->rc_rec, &c->rc_Z, &c->rc_GT, &c->in_soff, &c->in_sbytes, &c->long_h,
                    &c->long_which, &c->long_plane, &c->long_flags, &c->ra_S, &c->ra_St, &c->ra_rec, &c->ra_flag, &c->ra_Z, &c->ra_GT, &c->ev, &c->ev_n,
                    &c->pfl_chunks, &c->pfl_S, &c->pfl_C, &c->pfl_rc, &c->rt_cnt, &c->pfl_rec, &c->pfl_bk, &c->pfl_bv,
                    &c->pfl_ovf, &c->pfl_order})
        b->release();
    for (auto &ps : c->pfs) {
        for (DBuf *b : {&ps.chunks, &ps.rep, &ps.S, &ps.big_k, &ps.big_v, &ps.ovf}) b->release();
        if (ps.hashed) (void)hipEventDestroy(ps.hashed);
        if (ps.applied) (void)hipEventDestroy(ps.applied);
    }
    if (c->ev_w) (void)hipEventDestroy(c->ev_w);
    if (c->ev_r) (void)hipEventDestroy(c->ev_r);
    if (c->st2) (void)hipStreamDestroy(c->st2);
    if (c->st3) (void)hipStreamDestroy(c->st3);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
    return SK_OK;
}

const char *sk_last_error(sk_ctx *c) { return c ? c->err.c_str() : "no context"; }
void *sk_stream(sk_ctx *c) { return c ? (void *)c->st : nullptr; }
int sk_sync(sk_ctx *c) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    return sync(c);
}

int sk_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

uint32_t sk_crc16(const uint8_t *p, uint64_t len) {
    // CRC16-XMODEM: poly 0x1021, init 0 (M:connection/CRC16.java:23-61)
    static uint16_t table[256];
    static bool init = false;
    if (!init) {
        for (int i = 0; i < 256; i++) {
            uint16_t crc = uint16_t(i << 8);
            for (int b = 0; b < 8; b++) crc = (crc & 0x8000) ? uint16_t((crc << 1) ^ 0x1021) : uint16_t(crc << 1);
            table[i] = crc;
        }
        init = true;
    }
    uint32_t crc = 0;
    for (uint64_t i = 0; i < len; i++) crc = ((crc << 8) ^ table[((crc >> 8) ^ p[i]) & 0xff]) & 0xffff;
    return crc;
}

int32_t sk_calc_slot(const uint8_t *key, uint64_t len) {
    if (!key) return 0;
    const uint8_t *b = static_cast<const uint8_t *>(memchr(key, '{', len));
    if (b) {
        const uint8_t *e = static_cast<const uint8_t *>(memchr(key, '}', len)); // first '}' anywhere
        if (!e || e < b + 1) return -1; // Java substring() throws
        return int32_t(sk_crc16(b + 1, uint64_t(e - b - 1)) % 16384);
    }
    return int32_t(sk_crc16(key, len) % 16384);
}

int32_t sk_owner(const uint8_t *key, uint64_t len, int32_t n_gpus) {
    int32_t s = sk_calc_slot(key, len);
    if (s < 0 || n_gpus <= 0) return -1;
    return s % n_gpus;
}

int sk_owner_many(uint32_t n, const uint64_t *off, const uint8_t *bytes, int32_t n_gpus, int32_t *out) {
    for (uint32_t i = 0; i < n; i++) out[i] = sk_owner(bytes + off[i], off[i + 1] - off[i], n_gpus);
    return SK_OK;
}

int64_t sk_bloom_optimal_bits(int64_t n, double p) {
    if (p == 0) p = 4.9e-324; // Double.MIN_VALUE
    double v = double(-n) * std::log(p) / (std::log(2) * std::log(2));
    if (v != v) return 0;
    if (v >= 9.2233720368547758e18) return INT64_MAX;
    if (v <= -9.2233720368547758e18) return INT64_MIN;
    return int64_t(v);
}

int32_t sk_bloom_optimal_k(int64_t n, int64_t m) {
    double x = double(m) / double(n) * std::log(2);
    double r = std::floor(x + 0.5); // Math.round
    int64_t l = (r != r) ? 0 : (r >= 9.2233720368547758e18 ? INT64_MAX : int64_t(r));
    int32_t k = int32_t(l); // (int) of a long: low 32 bits
    return std::max(1, k);
}

uint64_t sk_hll_estimate_hist(const uint32_t *hist, int redis_major) {
    if (redis_major >= 5) return estimate_v5(hist);
    double E = 0;
    for (int v = 0; v < 64; v++) E += double(hist[v]) * g_pe[v];
    return estimate_v3(E, int(hist[0]));
}

// types of n keys in one call (the group-commit coalescers' check of the keys they have no cached slab id for)
int sk_type_many(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes, int32_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    for (uint32_t i = 0; i < n; i++) {
        std::string k = key_of(bytes + off[i], off[i + 1] - off[i]);
        auto it = c->keys.find(k);
        out[i] = it != c->keys.end() ? int32_t(it->second.type) : (c->bloom.count(k) ? 3 : SK_TYPE_NONE);
    }
    return SK_OK;
}

int sk_type(sk_ctx *c, const uint8_t *key, uint64_t len, int *out) {
    std::lock_guard<std::mutex> g(c->mu);
    std::string k = key_of(key, len);
    auto it = c->keys.find(k);
    if (it != c->keys.end()) *out = it->second.type;
    else *out = c->bloom.count(k) ? 3 : SK_TYPE_NONE;
    return SK_OK;
}

int sk_del(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes, uint64_t *removed) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint64_t cnt = 0;
    for (uint32_t i = 0; i < n; i++) {
        bool r;
        int rc = del_key(c, key_at(off, bytes, i), &r);
        if (rc) return rc;
        cnt += r;
    }
    if (removed) *removed = cnt;
    return sync(c);
}

// FLUSHALL / FLUSHDB: every key (HLL slabs re-zeroed and reused, strings
// freed) and every Bloom config
// pinned host memory for callers that fill their inputs in place (the JNI side's direct ByteBuffers): H2D from it
// runs at the link's rate with no staging copy
int sk_host_alloc(sk_ctx *c, uint64_t bytes, void **out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    *out = nullptr;
    HIPCHK(c, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return SK_OK;
}
int sk_host_free(sk_ctx *c, void *p) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (p) HIPCHK(c, hipHostFree(p));
    return SK_OK;
}

int sk_hll_epoch(sk_ctx *c, uint64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    *out = c->hll_epoch;
    return SK_OK;
}

int sk_flushall(sk_ctx *c) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::vector<std::string> names;
    names.reserve(c->keys.size());
    for (auto &kv : c->keys) names.push_back(kv.first);
    for (auto &k : names) {
        bool r;
        int rc = del_key(c, k, &r);
        if (rc) return rc;
    }
    c->bloom.clear();
    return sync(c);
}

static void find_hlls_parallel(sk_ctx *c, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes,
                               uint32_t *ids, uint8_t *found);

int sk_hll_resolve(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes, uint32_t *ids,
                   uint8_t *created) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    for (uint32_t i = 0; i < n; i++) {
        bool cr;
        int r = hll_get(c, key_at(off, bytes, i), true, &ids[i], &cr);
        if (r) return r;
        ids[i] = hll_handle(c, ids[i]);
        if (created) created[i] = cr;
    }
    return sync(c);
}

// HLL handles of existing keys without creating any (0xffffffff: no such key) -- what PFCOUNT / countWith read
// (a key holding a plain bit string is refused with WRONGTYPE, a valid HLL string is adopted, as PFCOUNT does)
int sk_hll_lookup(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes, uint32_t *ids) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::vector<uint8_t> found(n, 0);
    find_hlls_parallel(c, n, off, bytes, ids, found.data());
    for (uint32_t i = 0; i < n; i++) {
        uint32_t id;
        if (!found[i]) {
            int r = hll_get(c, key_at(off, bytes, i), false, &id, nullptr);
            if (r) return r;
        } else {
            id = ids[i];
        }
        ids[i] = id == kNoId ? kNoId : hll_handle(c, id);
    }
    return sync(c);
}

// ---------------------------------------------------------------- PFADD
// PFADD of commands whose keys are resolved (cmd_key[i], valid[i] = 0 skips a
// failed command; valid == nullptr: all valid): device batches of <= max_batch elements, replies in
// out_changed.  A chunk of valid one-element commands (the RBatch of add)
// ships the caller's ids, rebased offsets and bytes as they are; otherwise
// the valid commands' elements are re-packed with a command index each.
// distinct sketches of a batch: only the density heuristic of the non-default paths (pfadd_uses_sort) uses it, so
// the default partition path skips the count
static uint64_t pfadd_touched(const sk_ctx *c, const uint32_t *ids, uint64_t m) {
    if (c->pfadd_path == 1) return 0;
    std::vector<uint32_t> uniq(ids, ids + m);
    std::sort(uniq.begin(), uniq.end());
    return uint64_t(std::unique(uniq.begin(), uniq.end()) - uniq.begin());
}

static int pfadd_host_batch(sk_ctx *c, uint32_t n_cmds, const uint32_t *cmd_key, const uint8_t *valid,
                            const uint32_t *elem_counts, const uint64_t *elem_off, const uint8_t *elem_bytes,
                            uint8_t *out_changed) {
    std::memset(out_changed, 0, n_cmds);
    // element index of command i's first element (cmd_e0[i] = i when every command has one element)
    bool all_one = true;
    for (uint32_t i = 0; i < n_cmds && all_one; i++) all_one = elem_counts[i] == 1;
    std::vector<uint64_t> &e0v = c->h_e0;
    if (!all_one) {
        e0v.resize(n_cmds + 1);
        uint64_t total_e = 0;
        for (uint32_t i = 0; i < n_cmds; i++) {
            e0v[i] = total_e;
            total_e += elem_counts[i];
        }
        e0v[n_cmds] = total_e;
    }
    auto cmd_e0 = [&](uint32_t i) -> uint64_t { return all_one ? uint64_t(i) : e0v[i]; };
    uint32_t c0 = 0;
    std::vector<uint32_t> h_ids, h_cmd;
    std::vector<uint64_t> &off2 = c->h_off;
    std::vector<uint8_t> bytes2;
    while (c0 < n_cmds) {
        // commands [c0, c1) -- a single command larger than max_batch goes alone
        uint32_t c1 = c0;
        uint64_t ne = 0;
        bool simple = true; // every command valid with one element
        if (all_one && !valid) { // every command valid with one element: chunk by count
            c1 = uint32_t(std::min<uint64_t>(n_cmds, uint64_t(c0) + std::max<uint64_t>(c->max_batch, 1)));
        } else {
            while (c1 < n_cmds && (c1 == c0 || ne + elem_counts[c1] <= c->max_batch)) {
                simple = simple && (!valid || valid[c1]) && elem_counts[c1] == 1;
                ne += elem_counts[c1++];
            }
        }
        uint64_t e0 = cmd_e0(c0), b0 = elem_off[e0], b1 = elem_off[cmd_e0(c1)];
        const uint32_t *ids_src, *cmd_src = nullptr;
        const uint64_t *off_src;
        const uint8_t *bytes_src;
        uint64_t m, nbytes, shift = 0; // simple chunks: the caller's offsets as they are, the bytes from b0 down to
                                       // a 16-B boundary, and the device byte pointer moved back by that base
        if (!simple) off2.clear();
        if (simple) {
            m = c1 - c0;
            shift = b0 & ~uint64_t(15);
            off_src = elem_off + e0;
            ids_src = cmd_key + c0;
            bytes_src = elem_bytes + shift;
            nbytes = b1 - shift;
        } else {
            h_ids.clear();
            h_cmd.clear();
            bytes2.clear();
            uint64_t t = 0;
            for (uint32_t cc = c0; cc < c1; cc++) {
                if (valid && !valid[cc]) continue;
                for (uint64_t e = cmd_e0(cc); e < cmd_e0(cc + 1); e++) {
                    uint64_t l = elem_off[e + 1] - elem_off[e];
                    h_ids.push_back(cmd_key[cc]);
                    h_cmd.push_back(cc - c0);
                    off2.push_back(t);
                    bytes2.insert(bytes2.end(), elem_bytes + elem_off[e], elem_bytes + elem_off[e] + l);
                    t += l;
                }
            }
            off2.push_back(t);
            m = h_ids.size();
            off_src = off2.data();
            ids_src = h_ids.data();
            cmd_src = h_cmd.data();
            bytes_src = bytes2.data();
            nbytes = t;
        }
        static const bool tdbg = getenv("SK_HOST_TIMING") != nullptr; // dev knob: phase times to stderr
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto t0 = now();
        if (m) {
            HIPCHK(c, c->in_ids.ensure(m * 4));
            HIPCHK(c, c->in_off.ensure((m + 1) * 8));
            HIPCHK(c, c->in_bytes.ensure(nbytes + 16));
            HIPCHK(c, c->out_u8.ensure(c1 - c0));
            int sr;
            if ((sr = stage_h2d(c, c->in_ids.p, ids_src, m * 4))) return sr;
            if (cmd_src) {
                HIPCHK(c, c->in_cmd.ensure(m * 4));
                if ((sr = stage_h2d(c, c->in_cmd.p, cmd_src, m * 4))) return sr;
            }
            if ((sr = stage_h2d(c, c->in_off.p, off_src, (m + 1) * 8))) return sr;
            if ((sr = stage_h2d(c, c->in_bytes.p, bytes_src, nbytes))) return sr;
            HIPCHK(c, hipMemsetAsync(c->in_bytes.as<uint8_t>() + nbytes, 0, 16, c->st)); // padding contract
            HIPCHK(c, hipMemsetAsync(c->out_u8.p, 0, c1 - c0, c->st));
            const uint64_t touched = pfadd_touched(c, ids_src, m);
            // long elements (addAll's Q1 element: the whole Jackson array) are hashed by one workgroup each
            const uint64_t *d_pre = nullptr;
            if (c->pfadd_path == 1 && nbytes >= sk::long_elem_bytes()) {
                std::vector<uint32_t> which, first_wg{0};
                std::vector<uint64_t> poff{0};
                for (uint64_t j = 0; j < m; j++)
                    if (off_src[j + 1] - off_src[j] >= sk::long_elem_bytes()) {
                        which.push_back(uint32_t(j));
                        first_wg.push_back(first_wg.back() + sk::murmur_long_wgs(off_src[j + 1] - off_src[j]));
                        poff.push_back(poff.back() + sk::murmur_long_plane_words(off_src[j + 1] - off_src[j]));
                    }
                if (!which.empty()) {
                    const uint32_t nl = uint32_t(which.size()), nwg = first_wg.back();
                    which.insert(which.end(), first_wg.begin(), first_wg.end());
                    if (which.size() & 1) which.push_back(0); // poff starts at an even word
                    const size_t at = which.size();
                    which.resize(at + 2 * poff.size());
                    std::memcpy(which.data() + at, poff.data(), poff.size() * 8);
                    HIPCHK(c, c->long_h.ensure(m * 8));
                    HIPCHK(c, c->long_which.ensure(which.size() * 4));
                    HIPCHK(c, c->long_plane.ensure(poff.back() * 4));
                    HIPCHK(c, c->long_flags.ensure((uint64_t(nwg) * 64 + 2) * 4));
                    HIPCHK(c, hipMemcpyAsync(c->long_which.p, which.data(), which.size() * 4, hipMemcpyHostToDevice,
                                             c->st));
                    { Prof p_(c, 21);
                    HIPCHK(c, sk::launch_murmur_long(c->st, nl, nwg, c->in_bytes.as<uint8_t>() - shift,
                                                     c->in_off.as<uint64_t>(), c->long_which.as<uint32_t>(),
                                                     c->long_plane.as<uint32_t>(), c->long_flags.as<uint32_t>(),
                                                     c->long_h.as<uint64_t>())); }
                    uint32_t lerr = 0;
                    HIPCHK(c, hipMemcpyAsync(&lerr, c->long_flags.as<uint32_t>() + uint64_t(nwg) * 64 + 1, 4,
                                             hipMemcpyDeviceToHost, c->st));
                    HIPCHK(c, hipStreamSynchronize(c->st)); // `which` is a host vector
                    // a look-back wait that ran out (a predecessor workgroup delayed, e.g. on a shared GPU) leaves
                    // these hashes invalid: the hash kernels then hash the long elements per thread instead (slow,
                    // no waits), so the call still succeeds
                    c->long_fallbacks += lerr ? 1 : 0;
                    d_pre = lerr ? nullptr : c->long_h.as<uint64_t>();
                }
            }
            int r = pfadd_device(c, m, c->in_ids.as<uint32_t>(), c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>() - shift,
                                 cmd_src ? c->in_cmd.as<uint32_t>() : nullptr, c1 - c0, c->out_u8.as<uint8_t>(),
                                 touched, d_pre);
            if (r) return r;
            auto t1 = now();
            HIPCHK(c, hipMemcpyAsync(out_changed + c0, c->out_u8.p, c1 - c0, hipMemcpyDeviceToHost, c->st));
            r = sync(c);
            if (r) return r;
            if (tdbg)
                fprintf(stderr, "[sk host pfadd] m=%llu enqueue %.3f ms, d2h+sync %.3f ms\n", (unsigned long long)m,
                        std::chrono::duration<double, std::milli>(t1 - t0).count(),
                        std::chrono::duration<double, std::milli>(now() - t1).count());
        }
        c0 = c1;
    }
    return SK_OK;
}

// Parallel read-only pass over the key directory for a large batch: found[i] =
// 1 and ids[i] set where key i already names an HLL.  Everything else (new
// keys, strings to adopt, wrong types) is left to the caller's in-order pass,
// so creation order and error text are those of the serial lookup.
static void find_hlls_parallel(sk_ctx *c, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes,
                               uint32_t *ids, uint8_t *found) {
    if (n < 65536 || HostPool::get().threads() == 1) return;
    auto work = [&](uint64_t i0, uint64_t i1) {
        std::string k;
        for (uint32_t i = i0; i < i1; i++) {
            k.assign(reinterpret_cast<const char *>(key_bytes + key_off[i]), key_off[i + 1] - key_off[i]);
            auto it = c->keys.find(k);
            if (it != c->keys.end() && it->second.type == SK_TYPE_HLL) {
                ids[i] = it->second.id;
                found[i] = 1;
            }
        }
    };
    host_for(n, 4096, work);
}

int sk_pfadd(sk_ctx *c, uint32_t n_cmds, const uint64_t *key_off, const uint8_t *key_bytes,
             const uint32_t *elem_counts, const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out_changed) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n_cmds) return SK_OK;
    // resolve keys in command order; the first command on a created key replies 1
    std::vector<uint32_t> cmd_key(n_cmds);
    std::vector<uint8_t> first_created(n_cmds, 0);
    int status = SK_OK;
    std::vector<uint8_t> valid(n_cmds, 1), found(n_cmds, 0);
    find_hlls_parallel(c, n_cmds, key_off, key_bytes, cmd_key.data(), found.data());
    std::string k;
    for (uint32_t i = 0; i < n_cmds; i++) {
        if (found[i]) continue;
        bool cr;
        k.assign(reinterpret_cast<const char *>(key_bytes + key_off[i]), key_off[i + 1] - key_off[i]);
        int r = hll_get(c, k, true, &cmd_key[i], &cr);
        if (r == SK_EWRONGTYPE || r == SK_ECORRUPT) { // that command alone fails, as in a pipeline
            valid[i] = 0;
            status = r;
            continue;
        }
        if (r) return r;
        if (cr) first_created[i] = 1;
    }
    int r = pfadd_host_batch(c, n_cmds, cmd_key.data(), status == SK_OK ? nullptr : valid.data(), elem_counts,
                             elem_off, elem_bytes, out_changed);
    if (r) return r;
    for (uint32_t i = 0; i < n_cmds; i++)
        if (first_created[i]) out_changed[i] = 1;
    return status;
}

int sk_pfadd_ids(sk_ctx *c, uint32_t n_cmds, const uint32_t *key_ids, const uint32_t *elem_counts,
                 const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out_changed) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n_cmds) return SK_OK;
    const uint64_t d = first_dead_handle(c, n_cmds, key_ids);
    if (d < n_cmds)
        return fail(c, SK_ESTALE, "PFADD: slab id %u is not held by a key (deleted, replaced or never resolved)",
                    key_ids[d]);
    return pfadd_host_batch(c, n_cmds, key_ids, nullptr, elem_counts, elem_off, elem_bytes, out_changed);
}

int sk_pfadd_dev(sk_ctx *c, uint64_t n, const uint32_t *d_ids, const uint64_t *d_off, const uint8_t *d_bytes,
                 uint64_t bytes_len, uint8_t *d_changed) {
    (void)bytes_len;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device)); // touches only the HLL arena: no wait on the read stream
    if (c->pf_pending) {
        int r = pfadd_settle(c);
        if (r) return r;
    }
    if (!n) return SK_OK;
    unsigned id_bits = bits_for(c->hll_next ? c->hll_next - 1 : 0);
    uint64_t max_cmds = std::min<uint64_t>(c->max_batch, 1ull << std::min(32u, 64 - 20 - id_bits));
    struct DevCall { // the pipelined partition path is for caller-owned device inputs only
        sk_ctx *c;
        explicit DevCall(sk_ctx *c_) : c(c_) { c->pf_dev_call = true; }
        ~DevCall() { c->pf_dev_call = false; }
    } dev_call(c);
    if (pfadd_lines_ok(c, n)) { // group-committed RBatches: the line schedule, 2^26 elements per call
        for (uint64_t s = 0; s < n; s += (1ull << 26)) {
            uint64_t m = std::min<uint64_t>(1ull << 26, n - s);
            Prof p_(c, 20);
            int r = pfadd_lines(c, m, d_ids + s, d_off + s, d_bytes, d_changed + s);
            if (r) return r;
        }
        return c->async_dev ? SK_OK : sync(c);
    }
    for (uint64_t s = 0; s < n; s += max_cmds) {
        uint64_t m = std::min(max_cmds, n - s);
        Prof p_(c, 20); // the whole PFADD chain of this batch
        int r = pfadd_device(c, m, d_ids + s, d_off + s, d_bytes, nullptr, m, d_changed + s, 0);
        if (r) return r;
    }
    return c->async_dev ? SK_OK : sync(c);
}

// --------------------------------------------------------------- PFCOUNT
int sk_hll_sum_dev(sk_ctx *c, uint64_t n, const uint32_t *d_ids, uint64_t *d_out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    { Prof p_(c, 27);
    HIPCHK(c, sk::launch_hll_sum(c->st, n, d_ids, c->arena, d_out)); }
    return sync(c);
}

int sk_hll_histogram_dev(sk_ctx *c, uint64_t n, const uint32_t *d_ids, uint32_t *d_hist) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    { Prof p_(c, 3);
    HIPCHK(c, sk::launch_hll_hist(c->st, n, d_ids, c->arena, d_hist, 1)); }
    return sync(c);
}

// Single-key counts under the 3.x estimator from the device's exact register sums (k_hll_sum): E = S * 2^-40 when
// no register is >= 40 (bit-identical to hllDenseSum, see the kernel), else Redis's register-order sum.
static int estimate_many_sums(sk_ctx *c, uint64_t n, const uint64_t *s2, const uint32_t *ids, int64_t *out) {
    std::vector<uint8_t> slow(n, 0);
    auto work = [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; i++) {
            const uint32_t zeros = uint32_t(s2[2 * i + 1]), ge40 = uint32_t(s2[2 * i + 1] >> 32);
            if (!ge40) out[i] = int64_t(estimate_v3(std::ldexp(double(s2[2 * i]), -40), int(zeros)));
            else slow[i] = 1;
        }
    };
    host_for(n, 32768, work);
    for (uint64_t i = 0; i < n; i++) {
        if (!slow[i]) continue;
        std::vector<uint8_t> regs(kHllBytes), body(kSlabBytes);
        HIPCHK(c, hipMemcpy(body.data(), c->arena + uint64_t(ids[i] & kSlabMask) * kSlabBytes, kSlabBytes,
                            hipMemcpyDeviceToHost));
        hll_body_unpack(body.data(), regs.data());
        int ez;
        const double E = dense_sum(regs.data(), &ez);
        out[i] = int64_t(estimate_v3(E, ez));
    }
    return SK_OK;
}
int hll_sums(sk_ctx *c, uint64_t n, const uint32_t *d_ids, std::vector<uint64_t> &s2) {
    HIPCHK(c, c->hist.ensure(n * 16));
    { Prof p_(c, 27);
    HIPCHK(c, sk::launch_hll_sum(c->st, n, d_ids, c->arena, c->hist.as<uint64_t>())); }
    s2.resize(n * 2);
    HIPCHK(c, hipMemcpyAsync(s2.data(), c->hist.p, n * 16, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

// Estimates of many single-key counts from 64-bin histograms: exact-sum histograms (every register < 40, and every
// redis >= 5 estimate) in parallel threads, the rest (the register-order sum needs a register readback) in order
// afterwards.
static int estimate_many(sk_ctx *c, uint64_t n, const uint32_t *h, const uint32_t *ids, int64_t *out) {
    std::vector<uint8_t> slow(n, 0);
    auto work = [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; i++) {
            const uint32_t *hi = h + i * 64;
            if (c->redis_major >= 5) {
                out[i] = int64_t(estimate_v5(hi));
            } else if (hist_exact_v3(hi)) {
                double E = 0;
                for (int v = 0; v < 64; v++) E += double(hi[v]) * g_pe[v];
                out[i] = int64_t(estimate_v3(E, int(hi[0])));
            } else {
                slow[i] = 1;
            }
        }
    };
    host_for(n, 16384, work);
    for (uint64_t i = 0; i < n; i++) {
        if (!slow[i]) continue;
        int rc;
        out[i] = int64_t(
            estimate_host(c, h + i * 64, c->arena + uint64_t(ids[i] & kSlabMask) * kSlabBytes, false, &rc, true));
        if (rc) return rc;
    }
    return SK_OK;
}

int sk_pfcount_ids(sk_ctx *c, uint64_t n, const uint32_t *key_ids, int64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    const uint64_t d = first_dead_handle(c, n, key_ids);
    if (d < n)
        return fail(c, SK_ESTALE, "PFCOUNT: slab id %u is not held by a key (deleted, replaced or never resolved)",
                    key_ids[d]);
    HIPCHK(c, c->in_ids.ensure(n * 4));
    HIPCHK(c, hipMemcpyAsync(c->in_ids.p, key_ids, n * 4, hipMemcpyHostToDevice, c->st));
    int r2;
    if (c->redis_major < 5) { // exact register sums on the device (k_hll_sum)
        std::vector<uint64_t> s2;
        int r = hll_sums(c, n, c->in_ids.as<uint32_t>(), s2);
        if (r) return r;
        r2 = estimate_many_sums(c, n, s2.data(), key_ids, out);
    } else {
        std::vector<uint32_t> h;
        int r = hll_histograms(c, n, c->in_ids.as<uint32_t>(), c->arena, h);
        if (r) return r;
        r2 = estimate_many(c, n, h.data(), key_ids, out);
    }
    if (r2 || !c->hll_exact) return r2;
    for (uint64_t i = 0; i < n; i++) hll_card_cache(c, key_ids[i] & kSlabMask, &out[i]);
    return SK_OK;
}

int sk_pfcount(sk_ctx *c, uint32_t n_cmds, const uint32_t *nkeys, const uint64_t *key_off, const uint8_t *key_bytes,
               int64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    // single-key commands: one histogram launch over all of them
    std::vector<uint32_t> single_ids;
    std::vector<uint32_t> single_cmd;
    uint64_t k = 0;
    int status = SK_OK;
    std::vector<std::vector<uint32_t>> multi(n_cmds);
    std::vector<uint8_t> is_multi(n_cmds, 0), bad(n_cmds, 0);
    uint64_t total_keys = 0;
    for (uint32_t cmd = 0; cmd < n_cmds; cmd++) total_keys += nkeys[cmd];
    std::vector<uint32_t> fids;
    std::vector<uint8_t> found;
    if (total_keys >= 65536 && total_keys < (1ull << 32)) { // existing HLLs in a parallel read-only pass
        fids.resize(total_keys);
        found.assign(total_keys, 0);
        find_hlls_parallel(c, uint32_t(total_keys), key_off, key_bytes, fids.data(), found.data());
    }
    std::string kb;
    std::vector<uint32_t> ids;
    for (uint32_t cmd = 0; cmd < n_cmds; cmd++) {
        out[cmd] = 0;
        ids.clear();
        for (uint32_t j = 0; j < nkeys[cmd]; j++, k++) {
            uint32_t id;
            int r = SK_OK;
            if (!found.empty() && found[k]) {
                id = fids[k];
            } else {
                kb.assign(reinterpret_cast<const char *>(key_bytes + key_off[k]), key_off[k + 1] - key_off[k]);
                r = hll_get(c, kb, false, &id, nullptr);
            }
            if (r == SK_EWRONGTYPE || r == SK_ECORRUPT) { // that command alone fails, as in a pipeline
                bad[cmd] = 1;
                status = r;
                continue;
            }
            if (r) return r;
            if (id != kNoId) ids.push_back(id);
        }
        if (bad[cmd]) continue;
        if (nkeys[cmd] == 1) {
            if (!ids.empty()) {
                single_ids.push_back(ids[0]);
                single_cmd.push_back(cmd);
            }
        } else {
            is_multi[cmd] = 1;
            multi[cmd] = ids;
        }
    }
    std::vector<uint32_t> h;
    if (!single_ids.empty()) {
        HIPCHK(c, c->in_ids.ensure(single_ids.size() * 4));
        HIPCHK(c, hipMemcpyAsync(c->in_ids.p, single_ids.data(), single_ids.size() * 4, hipMemcpyHostToDevice, c->st));
        std::vector<int64_t> est(single_ids.size());
        int r;
        if (c->redis_major < 5) { // exact register sums on the device (k_hll_sum)
            std::vector<uint64_t> s2;
            if ((r = hll_sums(c, single_ids.size(), c->in_ids.as<uint32_t>(), s2))) return r;
            if ((r = estimate_many_sums(c, single_ids.size(), s2.data(), single_ids.data(), est.data()))) return r;
        } else {
            if ((r = hll_histograms(c, single_ids.size(), c->in_ids.as<uint32_t>(), c->arena, h))) return r;
            if ((r = estimate_many(c, single_ids.size(), h.data(), single_ids.data(), est.data()))) return r;
        }
        for (size_t i = 0; i < single_ids.size(); i++) {
            out[single_cmd[i]] = est[i];
            hll_card_cache(c, single_ids[i], &out[single_cmd[i]]);
        }
    }
    // multi-key commands: union into a temporary raw register array (nothing modified)
    HIPCHK(c, c->uni.ensure(kHllBytes));
    HIPCHK(c, c->misc.ensure(4096));
    for (uint32_t cmd = 0; cmd < n_cmds; cmd++) {
        if (!is_multi[cmd]) continue;
        int r = union_into(c, multi[cmd], c->uni.as<uint8_t>(), 0, 0);
        if (r) return r;
        r = hll_histograms(c, 1, c->d_zero, c->uni.as<uint8_t>(), h);
        if (r) return r;
        int rc;
        out[cmd] = int64_t(estimate_host(c, h.data(), c->uni.as<uint8_t>(), true, &rc));
        if (rc) return rc;
    }
    return status;
}

// PFCOUNT of a raw register array in device memory, multi-key semantics (hllCount over the temporary raw
// registers of pfcountCommand): the last step of a cross-GPU countWith after the MAX all-reduce, with no key
int sk_hll_count_registers_dev(sk_ctx *c, const uint8_t *d_regs, int64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::vector<uint32_t> h;
    int r = hll_histograms(c, 1, c->d_zero, d_regs, h);
    if (r) return r;
    int rc;
    *out = int64_t(estimate_host(c, h.data(), d_regs, true, &rc));
    return rc;
}

int sk_hll_union_dev(sk_ctx *c, uint64_t n, const uint32_t *d_ids, uint8_t *d_out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    const uint64_t max_groups = 4096;
    HIPCHK(c, c->partial.ensure((max_groups + max_groups / 64 + 2) * kHllBytes));
    { Prof p_(c, 4);
    HIPCHK(c, sk::launch_hll_union(c->st, n, d_ids, c->arena, c->partial.as<uint8_t>(), max_groups, d_out, 0, 1, 0)); }
    return sync(c);
}

// The local step of a countWith / PFMERGE over keys sharded by calcSlot % n_gpus (redisson_amd/cluster.py):
// register max of the existing HLLs among `keys` that this rank owns, into d_out (16384 B on the device).
// Owner filtering and the directory lookup run on host threads; *n_used = HLLs merged.
int sk_hll_union_keys(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes, int32_t n_gpus,
                      int32_t rank, uint8_t *d_out, uint32_t *n_used) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::vector<int32_t> own(n);
    {
        host_for(n, 32768, [&](uint64_t i0, uint64_t i1) {
            for (uint64_t i = i0; i < i1; i++) own[i] = sk_owner(bytes + off[i], off[i + 1] - off[i], n_gpus);
        });
    }
    std::vector<uint64_t> so(1, 0); // the owned keys, packed
    std::vector<uint8_t> sb;
    for (uint32_t i = 0; i < n; i++)
        if (own[i] == rank) {
            sb.insert(sb.end(), bytes + off[i], bytes + off[i + 1]);
            so.push_back(sb.size());
        }
    const uint32_t m = uint32_t(so.size() - 1);
    sb.resize(sb.size() + 16, 0);
    std::vector<uint32_t> ids(m);
    std::vector<uint8_t> found(m, 0);
    find_hlls_parallel(c, m, so.data(), sb.data(), ids.data(), found.data());
    uint32_t k = 0;
    for (uint32_t i = 0; i < m; i++) {
        uint32_t id = ids[i];
        if (!found[i]) {
            int r = hll_get(c, key_at(so.data(), sb.data(), i), false, &id, nullptr);
            if (r) return r;
        }
        if (id != kNoId) ids[k++] = id;
    }
    if (n_used) *n_used = k;
    if (!k) {
        HIPCHK(c, hipMemsetAsync(d_out, 0, kHllBytes, c->st));
        return sync(c);
    }
    HIPCHK(c, c->in_ids.ensure(uint64_t(k) * 4));
    HIPCHK(c, hipMemcpyAsync(c->in_ids.p, ids.data(), uint64_t(k) * 4, hipMemcpyHostToDevice, c->st));
    const uint64_t max_groups = 4096;
    HIPCHK(c, c->partial.ensure((max_groups + max_groups / 64 + 2) * kHllBytes));
    { Prof p_(c, 4);
    HIPCHK(c, sk::launch_hll_union(c->st, k, c->in_ids.as<uint32_t>(), c->arena, c->partial.as<uint8_t>(), max_groups,
                                   d_out, 0, 1, 0)); }
    return sync(c); // ids is a host vector
}

int sk_pfmerge(sk_ctx *c, const uint8_t *dest, uint64_t dest_len, uint32_t n_src, const uint64_t *src_off,
               const uint8_t *src_bytes) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    // check every source first (pfmergeCommand checks before touching dest)
    std::vector<uint32_t> ids;
    for (uint32_t i = 0; i < n_src; i++) {
        uint32_t id;
        int r = hll_get(c, key_at(src_off, src_bytes, i), false, &id, nullptr);
        if (r) return r;
        if (id != kNoId) ids.push_back(id);
    }
    uint32_t did;
    int r = hll_get(c, key_of(dest, dest_len), true, &did, nullptr);
    if (r) return r;
    hll_str_merged(c, did);
    return union_into(c, ids, c->arena + uint64_t(did) * kSlabBytes, 1, 1);
}

int sk_hll_merge_registers_dev(sk_ctx *c, const uint8_t *key, uint64_t len, const uint8_t *d_regs) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t did;
    int r = hll_get(c, key_of(key, len), true, &did, nullptr);
    if (r) return r;
    hll_str_merged(c, did);
    // out = max(out, d_regs): a one-key union whose "arena" is d_regs
    const uint64_t max_groups = 4096;
    HIPCHK(c, c->partial.ensure((max_groups + max_groups / 64 + 2) * kHllBytes));
    HIPCHK(c, sk::launch_hll_union(c->st, 1, c->d_zero, d_regs, c->partial.as<uint8_t>(), max_groups,
                                   c->arena + uint64_t(did) * kSlabBytes, 1, 0, 1));
    return sync(c);
}

int sk_hll_registers(sk_ctx *c, const uint8_t *key, uint64_t len, uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t id;
    int r = hll_get(c, key_of(key, len), false, &id, nullptr);
    if (r) return r;
    if (id == kNoId) {
        std::memset(out, 0, kHllBytes);
        return SK_OK;
    }
    std::vector<uint8_t> body(kSlabBytes);
    HIPCHK(c, hipMemcpyAsync(body.data(), c->arena + uint64_t(id) * kSlabBytes, kSlabBytes, hipMemcpyDeviceToHost, c->st));
    int rr = sync(c);
    if (!rr) hll_body_unpack(body.data(), out);
    return rr;
}

} // extern "C"

// ============================================================== bit strings
extern "C" {

} // extern "C"

namespace {
// The keys of a bit batch, each distinct key resolved once (RBatch SETBIT / GETBIT runs name one bitset over and over:
// a run of equal keys is found by comparing bytes, other repeats through a map of the batch's own key bytes)
struct BitKeys {
    bool single = true;           // every op names key 0
    std::vector<uint32_t> kid;    // per op (multi-key): its key's index
    std::vector<uint64_t> first;  // per key: an op naming it (its bytes)
};
// one parallel pass over a bit batch: does every op name op 0's key, are all offsets below `lim`, do all values
// equal values[0] (values may be null), the largest valid offset
struct BitScan {
    bool single = true, all_valid = true, one_value = true, any_valid = false;
    uint64_t mx = 0;
};
BitScan bit_scan(uint64_t n, const uint64_t *key_off, const uint8_t *key_bytes, const uint64_t *offs,
                 const uint8_t *values, uint64_t lim) {
    BitScan S;
    std::mutex mu;
    const uint64_t l0 = key_off[1] - key_off[0];
    const uint8_t v0 = values ? values[0] & 1u : 0u;
    host_for(n, 1u << 18, [&](uint64_t i0, uint64_t i1) {
        BitScan L;
        for (uint64_t i = i0; i < i1; i++) {
            L.single &= key_off[i + 1] - key_off[i] == l0 &&
                        std::memcmp(key_bytes + key_off[i], key_bytes + key_off[0], l0) == 0;
            if (values) L.one_value &= (values[i] & 1u) == v0;
            if (offs[i] >= lim) {
                L.all_valid = false;
            } else {
                L.mx = L.any_valid ? std::max(L.mx, offs[i]) : offs[i];
                L.any_valid = true;
            }
        }
        std::lock_guard<std::mutex> g(mu);
        S.single &= L.single;
        S.all_valid &= L.all_valid;
        S.one_value &= L.one_value;
        if (L.any_valid) S.mx = S.any_valid ? std::max(S.mx, L.mx) : L.mx;
        S.any_valid |= L.any_valid;
    });
    return S;
}
void bit_keys(uint64_t n, const uint64_t *key_off, const uint8_t *key_bytes, BitKeys &K, bool single) {
    K.single = single;
    K.first.assign(1, 0);
    if (K.single) return;
    K.kid.assign(n, 0);
    std::unordered_map<std::string_view, uint32_t> ix;
    auto view = [&](uint64_t i) {
        return std::string_view(reinterpret_cast<const char *>(key_bytes + key_off[i]), key_off[i + 1] - key_off[i]);
    };
    ix.emplace(view(0), 0u);
    for (uint64_t i = 1; i < n; i++) {
        if (key_off[i + 1] - key_off[i] == key_off[i] - key_off[i - 1] &&
            std::memcmp(key_bytes + key_off[i], key_bytes + key_off[i - 1], key_off[i + 1] - key_off[i]) == 0) {
            K.kid[i] = K.kid[i - 1]; // the same key as the op before
            continue;
        }
        auto it = ix.emplace(view(i), uint32_t(K.first.size()));
        if (it.second) K.first.push_back(i);
        K.kid[i] = it.first->second;
    }
}

// dense / sparse SETBIT_VOID of one value on string `id` (device offsets, max offset mx already validated and the
// string grown): a dense batch streams the string through LDS region by region (k_sbv_part / k_sbv_fine /
// k_sbv_runs) instead of one random atomic per op (k_setbit_void); the ops of one value commute
int setbit_void_device(sk_ctx *c, uint32_t id, uint64_t n, const uint64_t *d_offsets, uint64_t mx, uint8_t value) {
    const uint64_t need = (mx >> 3) + 1;
    const unsigned rb = sk::sbv_region_bits(), eb = 64u - unsigned(__builtin_clzll(mx | 1));
    const uint64_t nr = (mx >> rb) + 1; // regions up to the highest op; >= 256 of them to fill the GPU
    if (n >= c->sbv_min && n < (uint64_t(1) << 32) && n * 64 >= need && nr >= 256 && c->sbv_part &&
        sk::sbv_part_ok(n, mx)) { // the hand-written region partition
        HIPCHK(c, c->keys_b.ensure(sk::sbv_part_scratch_bytes(n, mx)));
        Prof p_(c, 9);
        HIPCHK(c, sk::launch_setbit_void_part(c->st, n, d_offsets, mx, c->keys_b.p, c->strs[id].ptr, c->strs[id].cap,
                                              value & 1));
    } else if (n >= c->sbv_min && n < (uint64_t(1) << 32) && n * 64 >= need && nr >= 256) {
        // the same through a radix sort of the offsets by region (SK_SBV_PART=0, or a call past the tables)
        const uint64_t *keys = d_offsets;
        HIPCHK(c, c->vals_a.ensure((nr + 1) * 4));
        Prof p_(c, 9);
        if (eb > rb) { // more than one region: group the ops by region
            size_t tmp;
            HIPCHK(c, sk::sort_keys_size(n, rb, eb, &tmp));
            HIPCHK(c, c->sort_tmp.ensure(tmp));
            HIPCHK(c, c->keys_b.ensure(n * 8));
            HIPCHK(c, sk::sort_keys(c->st, c->sort_tmp.p, c->sort_tmp.cap, d_offsets, c->keys_b.as<uint64_t>(), n, rb,
                                    eb));
            keys = c->keys_b.as<uint64_t>();
        }
        HIPCHK(c, sk::launch_setbit_void_regions(c->st, n, keys, mx, c->vals_a.as<uint32_t>(), c->strs[id].ptr,
                                                 c->strs[id].cap, value & 1));
    } else {
        Prof p_(c, 9);
        HIPCHK(c, sk::launch_setbit_void(c->st, n, d_offsets, c->strs[id].ptr, value & 1));
    }
    return SK_OK;
}

// SETBIT through the region partition with u64 records, in pieces of <= 2^30 ops run one after another (an op's
// seq is 31 bits; later pieces see earlier ones' bits, as batch order does).  seg (device) holds nseg SbrSeg.
int setbit_regions(sk_ctx *c, uint64_t n, const uint64_t *d_off, const uint32_t *d_vrb, const uint8_t *d_vals,
                   uint8_t value, uint64_t NRv, const void *d_seg, uint32_t nseg, uint8_t *d_out) {
    constexpr uint64_t kPiece = uint64_t(1) << 30;
    for (uint64_t s0 = 0; s0 < n; s0 += kPiece) {
        const uint64_t m = std::min(kPiece, n - s0);
        if (!sk::sbr_ok(m, NRv))
            return fail(c, SK_EINVAL, "SETBIT batch of %llu ops over %llu regions of 2^%u bits is past the region tables",
                        (unsigned long long)m, (unsigned long long)NRv, sk::sbv_region_bits());
        HIPCHK(c, c->keys_b.ensure(sk::sbr_scratch_bytes(m, NRv)));
        Prof p_(c, 9);
        HIPCHK(c, sk::launch_setbit_regions(c->st, m, d_off + s0, d_vrb ? d_vrb + s0 : nullptr,
                                            d_vals ? d_vals + s0 : nullptr, value & 1u, NRv, d_seg, nseg, c->keys_b.p,
                                            d_out ? d_out + s0 : nullptr));
    }
    return SK_OK;
}
// the same for one string (device batches): one segment
int setbit_regions_one(sk_ctx *c, uint32_t id, uint64_t n, const uint64_t *d_off, const uint8_t *d_vals, uint8_t value,
                       uint64_t mx, uint8_t *d_out) {
    const sk::SbrSegH one{0, c->strs[id].ptr, c->strs[id].cap};
    HIPCHK(c, c->ptrs.ensure(sizeof one));
    HIPCHK(c, hipMemcpyAsync(c->ptrs.p, &one, sizeof one, hipMemcpyHostToDevice, c->st));
    int r = setbit_regions(c, n, d_off, nullptr, d_vals, value, (mx >> sk::sbv_region_bits()) + 1, c->ptrs.p, 1, d_out);
    if (r) return r;
    return sync(c); // `one` is a stack variable
}

// grow string `id` to hold bit mx (capacity and length: SETBIT's sdsgrowzero)
int str_grow_bits(sk_ctx *c, uint32_t id, uint64_t mx) {
    const uint64_t need = (mx >> 3) + 1;
    uint64_t cur;
    int r = str_reserve(c, id, need);
    if (!r) r = str_len(c, id, &cur);
    if (!r && need > cur) r = str_set_len(c, id, need);
    return r;
}
} // namespace

extern "C" {

// SETBIT batch by key name (RBatch runs, RBitSet.set with a reply; M:RedissonBitSet.java:79-81,202-228).  Each
// distinct key is resolved once.  out_old == NULL is SETBIT_VOID (RBitSet.set(i), the Java executors pass no reply
// array for it): a batch of one key and one value takes the SETBIT_VOID kernels (the dense region path for a dense
// batch); everything else -- replies, several keys, mixed values -- the region partition with u64 records
// (k_sbv_part<u64> -> k_sbv_fine<u64> -> k_sbr_runs), whose replies are the bits as batch order finds them.  An op
// with a bad offset or on a key of another type fails alone (reply 0) and the call reports the error, as a pipeline.
int sk_setbit(sk_ctx *c, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, const uint64_t *offsets,
              const uint8_t *values, uint8_t *out_old) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    if (out_old) std::memset(out_old, 0, n);
    int status = SK_OK;
    const BitScan B = bit_scan(n, key_off, key_bytes, offsets, values, c->max_bit_offset);
    BitKeys K;
    bit_keys(n, key_off, key_bytes, K, B.single);
    const size_t nk = K.first.size();
    // per key: max valid offset
    std::vector<uint64_t> mx(nk, 0);
    std::vector<uint8_t> has(nk, 0);
    bool all_valid = B.all_valid;
    const bool one_value = B.one_value;
    const uint8_t v0 = values[0] & 1u;
    if (!all_valid) status = fail(c, SK_ERANGE, "%s", kRange);
    if (K.single) {
        mx[0] = B.mx;
        has[0] = B.any_valid;
    } else {
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t k = K.kid[i];
            if (offsets[i] >= c->max_bit_offset) continue;
            mx[k] = has[k] ? std::max(mx[k], offsets[i]) : offsets[i];
            has[k] = 1;
        }
    }
    // resolve / create each key once, grow its string; the call's virtual region space: one range per key
    std::vector<uint32_t> sid(nk, kNoId);
    std::vector<sk::SbrSegH> seg;
    std::vector<uint32_t> rbase(nk, 0xffffffffu);
    uint64_t NRv = 0;
    const unsigned RB = sk::sbv_region_bits();
    for (size_t k = 0; k < nk; k++) {
        if (!has[k]) continue;
        int r = str_get(c, key_at(key_off, key_bytes, K.first[k]), true, (mx[k] >> 3) + 1, &sid[k]);
        if (r == SK_EWRONGTYPE) {
            sid[k] = kNoId;
            all_valid = false;
            status = r;
            continue;
        }
        if (r || (r = str_grow_bits(c, sid[k], mx[k]))) return r;
        rbase[k] = uint32_t(std::min<uint64_t>(NRv, 0xfffffffeu));
        seg.push_back(sk::SbrSegH{NRv, c->strs[sid[k]].ptr, c->strs[sid[k]].cap});
        NRv += (mx[k] >> RB) + 1;
    }
    if (seg.empty()) return status;
    HIPCHK(c, c->in_off.ensure(uint64_t(n) * 8));
    HIPCHK(c, hipMemcpyAsync(c->in_off.p, offsets, uint64_t(n) * 8, hipMemcpyHostToDevice, c->st));
    if (!out_old && seg.size() == 1 && all_valid && one_value) { // SETBIT_VOID of one key and one value
        const uint32_t k = 0;
        int r = setbit_void_device(c, sid[k], n, c->in_off.as<uint64_t>(), mx[k], v0);
        if (r) return r;
        r = sync(c);
        return r ? r : status;
    }
    // per-op key bases (several keys, or ops to drop) and values (unless one value)
    const uint32_t *d_vrb = nullptr;
    const uint8_t *d_vals = nullptr;
    std::vector<uint32_t> vrb;
    if (!K.single || !all_valid) {
        vrb.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t k = K.single ? 0u : K.kid[i];
            vrb[i] = offsets[i] < c->max_bit_offset && sid[k] != kNoId ? rbase[k] : 0xffffffffu;
        }
        HIPCHK(c, c->in_ids.ensure(uint64_t(n) * 4));
        HIPCHK(c, hipMemcpyAsync(c->in_ids.p, vrb.data(), uint64_t(n) * 4, hipMemcpyHostToDevice, c->st));
        d_vrb = c->in_ids.as<uint32_t>();
    }
    if (!one_value) {
        HIPCHK(c, c->in_bytes.ensure(n));
        HIPCHK(c, hipMemcpyAsync(c->in_bytes.p, values, n, hipMemcpyHostToDevice, c->st));
        d_vals = c->in_bytes.as<uint8_t>();
    }
    HIPCHK(c, c->ptrs.ensure(seg.size() * sizeof(sk::SbrSegH)));
    HIPCHK(c, hipMemcpyAsync(c->ptrs.p, seg.data(), seg.size() * sizeof(sk::SbrSegH), hipMemcpyHostToDevice, c->st));
    uint8_t *d_out = nullptr;
    if (out_old) {
        HIPCHK(c, c->out_u8.ensure(n));
        HIPCHK(c, hipMemsetAsync(c->out_u8.p, 0, n, c->st));
        d_out = c->out_u8.as<uint8_t>();
    }
    int rr = setbit_regions(c, n, c->in_off.as<uint64_t>(), d_vrb, d_vals, v0, NRv, c->ptrs.p, uint32_t(seg.size()),
                            d_out);
    if (rr) {
        (void)sync(c);
        return rr;
    }
    if (out_old) HIPCHK(c, hipMemcpyAsync(out_old, d_out, n, hipMemcpyDeviceToHost, c->st));
    int r = sync(c); // vrb / offsets are host buffers
    return r ? r : status;
}

// GETBIT batch by key name: each distinct key resolved once; one key -> k_getbit_single on its string, several ->
// k_getbit_multi over per-op string ids.  Missing keys and bad offsets reply 0 (a bad offset also fails the call).
int sk_getbit(sk_ctx *c, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, const uint64_t *offsets,
              uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    int status = SK_OK;
    const BitScan B = bit_scan(n, key_off, key_bytes, offsets, nullptr, c->max_bit_offset);
    if (!B.all_valid) status = fail(c, SK_ERANGE, "%s", kRange); // such an op reads past the string: 0
    BitKeys K;
    bit_keys(n, key_off, key_bytes, K, B.single);
    std::vector<uint32_t> sid(K.first.size(), kNoId);
    for (size_t k = 0; k < K.first.size(); k++) {
        int r = str_get(c, key_at(key_off, key_bytes, K.first[k]), false, 0, &sid[k]);
        if (r == SK_EWRONGTYPE) {
            sid[k] = kNoId;
            status = r;
            continue;
        }
        if (r) return r;
    }
    HIPCHK(c, c->in_off.ensure(uint64_t(n) * 8));
    HIPCHK(c, c->out_u8.ensure(n));
    if (K.single && sid[0] == kNoId) {
        std::memset(out, 0, n);
        return status;
    }
    HIPCHK(c, hipMemcpyAsync(c->in_off.p, offsets, uint64_t(n) * 8, hipMemcpyHostToDevice, c->st));
    if (K.single) {
        Prof p_(c, 10);
        HIPCHK(c, sk::launch_getbit_single(c->st, n, c->in_off.as<uint64_t>(), c->strs[sid[0]].ptr,
                                           &c->d_dir[sid[0]].len, c->out_u8.as<uint8_t>()));
    } else {
        std::vector<uint32_t> ops(n);
        for (uint32_t i = 0; i < n; i++) ops[i] = sid[K.kid[i]];
        HIPCHK(c, c->in_ids.ensure(uint64_t(n) * 4));
        HIPCHK(c, hipMemcpyAsync(c->in_ids.p, ops.data(), uint64_t(n) * 4, hipMemcpyHostToDevice, c->st));
        Prof p_(c, 10);
        HIPCHK(c, sk::launch_getbit_multi(c->st, n, c->in_ids.as<uint32_t>(), c->in_off.as<uint64_t>(), c->d_dir,
                                          c->out_u8.as<uint8_t>()));
    }
    HIPCHK(c, hipMemcpyAsync(out, c->out_u8.p, n, hipMemcpyDeviceToHost, c->st));
    int r = sync(c);
    return r ? r : status;
}

// validate a device offset array: max offset -> host (one small readback)
static int dev_max_offset(sk_ctx *c, uint64_t n, const uint64_t *d_offsets, uint64_t *mx) {
    HIPCHK(c, sk::launch_max_u64(c->st, n, d_offsets, c->misc.as<uint64_t>()));
    HIPCHK(c, hipMemcpyAsync(mx, c->misc.p, 8, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_setbit_dev(sk_ctx *c, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets, uint8_t value,
                  uint8_t *d_out_old) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    uint64_t mx;
    int r = dev_max_offset(c, n, d_offsets, &mx);
    if (r) return r;
    if (mx >= c->max_bit_offset) return fail(c, SK_ERANGE, "%s", kRange);
    uint32_t id;
    if ((r = str_get(c, key_of(key, len), true, (mx >> 3) + 1, &id))) return r;
    uint64_t need = (mx >> 3) + 1, cur;
    if ((r = str_reserve(c, id, need))) return r;
    if ((r = str_len(c, id, &cur))) return r;
    if (need > cur && (r = str_set_len(c, id, need))) return r;
    if (!d_out_old) {
        if ((r = setbit_void_device(c, id, n, d_offsets, mx, value))) return r;
        return sync(c);
    }
    // replies: the region partition with the ops' seq (no library sort)
    return setbit_regions_one(c, id, n, d_offsets, nullptr, value, mx, d_out_old);
}

// Range-sharded RBitSet routing (cluster.py ShardedBitSet.set_dev / get_dev): a device batch of logical bit offsets
// split by owner shard (offset / shard_bits) into d_send -- shard 0's ops, then shard 1's, ..., each in batch order,
// as shard-local offsets (d_send_values alongside when d_values is given) -- and d_dst[i] = op i's slot there.
// out_counts[s] = ops for shard s (host).  An offset past the last shard fails the batch with SK_ERANGE.
int sk_route_bits(sk_ctx *c, uint64_t n, const uint64_t *d_offsets, const uint8_t *d_values, uint64_t shard_bits,
                  int32_t world, uint64_t *d_send, uint8_t *d_send_values, uint32_t *d_dst, uint64_t *out_counts) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (world <= 0 || uint32_t(world) > sk::route_max_world())
        return fail(c, SK_EINVAL, "route: world %d outside 1..%u", world, sk::route_max_world());
    if (!shard_bits) return fail(c, SK_EINVAL, "route: shard_bits is 0");
    if (n >= (1ull << 32)) return fail(c, SK_EINVAL, "route: batch of %llu ops (< 2^32)", (unsigned long long)n);
    for (int s = 0; s < world; s++) out_counts[s] = 0;
    if (!n) return SK_OK;
    const uint32_t nblk = sk::route_blocks(n);
    const uint64_t m = uint64_t(world) * nblk + 1;
    size_t tmp;
    HIPCHK(c, sk::route_scan_size(m, &tmp));
    HIPCHK(c, c->sort_tmp.ensure(std::max<size_t>(tmp, 16)));
    HIPCHK(c, c->rt_cnt.ensure(2 * m * 4));
    uint32_t *cnt = c->rt_cnt.as<uint32_t>(), *base = cnt + m;
    HIPCHK(c, hipMemsetAsync(cnt + (m - 1), 0, 4, c->st));
    HIPCHK(c, hipMemsetAsync(c->misc.p, 0, 4, c->st));
    HIPCHK(c, sk::launch_route(c->st, n, d_offsets, d_values, shard_bits, uint32_t(world), cnt, base, c->sort_tmp.p,
                               c->sort_tmp.cap, c->misc.as<uint32_t>(), d_send, d_send_values, d_dst));
    std::vector<uint32_t> b(world + 1);
    for (int s = 0; s <= world; s++)
        HIPCHK(c, hipMemcpyAsync(&b[s], base + uint64_t(s) * nblk, 4, hipMemcpyDeviceToHost, c->st));
    uint32_t bad = 0;
    HIPCHK(c, hipMemcpyAsync(&bad, c->misc.p, 4, hipMemcpyDeviceToHost, c->st));
    int r = sync(c);
    if (r) return r;
    if (bad) return fail(c, SK_ERANGE, "%s", kRange);
    for (int s = 0; s < world; s++) out_counts[s] = b[s + 1] - b[s];
    return SK_OK;
}

// replies of a routed batch back to batch order: d_out[i] = d_rep[d_dst[i]]
int sk_unroute_u8(sk_ctx *c, uint64_t n, const uint32_t *d_dst, const uint8_t *d_rep, uint8_t *d_out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    HIPCHK(c, sk::launch_unroute(c->st, n, d_dst, d_rep, d_out));
    return sync(c);
}

// The range-sharded Bloom filter's device steps (redisson_amd/cluster.py RangeShardedBloom): the probe indexes of
// a batch, routed like SETBIT / GETBIT, and the per-element reduction of the probes' replies
int sk_bloom_indexes_dev(sk_ctx *c, uint64_t n, const uint64_t *d_off, const uint8_t *d_bytes, int64_t size, int32_t k,
                         int32_t nprobe, uint64_t *d_idx) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (size <= 0 || k <= 0 || nprobe < 0 || nprobe > k)
        return fail(c, SK_EINVAL, "bloom indexes: size %lld, k %d, nprobe %d", (long long)size, k, nprobe);
    if (!n || !nprobe) return SK_OK;
    HIPCHK(c, sk::launch_bloom_indexes(c->st, n, d_off, d_bytes, uint64_t(size), magic_for(uint64_t(size)), nprobe,
                                       d_idx));
    return sync(c);
}
int sk_reduce_groups_u8(sk_ctx *c, uint64_t n, uint32_t group, uint32_t take, int invert, const uint8_t *d_in,
                        uint8_t *d_out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (take > group) return fail(c, SK_EINVAL, "reduce groups: take %u > group %u", take, group);
    HIPCHK(c, sk::launch_reduce_groups_u8(c->st, n, group, take, invert ? 1u : 0u, d_in, d_out));
    return sync(c);
}

// SETBIT of a device batch with one value per op (d_values u8[n]); replies (old bits) in d_out_old when given
int sk_setbit_values_dev(sk_ctx *c, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets,
                         const uint8_t *d_values, uint8_t *d_out_old) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    uint64_t mx;
    int r = dev_max_offset(c, n, d_offsets, &mx);
    if (r) return r;
    if (mx >= c->max_bit_offset) return fail(c, SK_ERANGE, "%s", kRange);
    uint32_t id;
    if ((r = str_get(c, key_of(key, len), true, (mx >> 3) + 1, &id))) return r;
    uint64_t need = (mx >> 3) + 1, cur;
    if ((r = str_reserve(c, id, need))) return r;
    if ((r = str_len(c, id, &cur))) return r;
    if (need > cur && (r = str_set_len(c, id, need))) return r;
    return setbit_regions_one(c, id, n, d_offsets, d_values, 0, mx, d_out_old);
}

// RBitSet.set(from, to) / clear(from, to): the reference sends one SETBIT_VOID
// per bit in one pipeline (M:RedissonBitSet.java:202-228).  Each SETBIT grows
// the string (sdsgrowzero) whatever the value; an out-of-range offset fails
// only its own command, so the in-range bits are applied and the call then
// reports SK_ERANGE, as the batch future would fail.
int sk_set_bit_range(sk_ctx *c, const uint8_t *key, uint64_t len, int64_t from, int64_t to, int value) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (from >= to) return SK_OK; // empty batch
    int64_t lim = int64_t(c->max_bit_offset);
    int64_t a = from < 0 ? 0 : from, b = to > lim ? lim : to;
    bool bad = from < 0 || to > lim;
    if (a < b) {
        uint64_t need = (uint64_t(b - 1) >> 3) + 1, cur;
        uint32_t id;
        int r = str_get(c, key_of(key, len), true, need, &id);
        if (r) return r;
        if ((r = str_reserve(c, id, need))) return r;
        if ((r = str_len(c, id, &cur))) return r;
        if (need > cur && (r = str_set_len(c, id, need))) return r;
        { Prof p_(c, 9);
        HIPCHK(c, sk::launch_bit_range(c->st, c->strs[id].ptr, uint64_t(a), uint64_t(b), value ? 1u : 0u)); }
        if ((r = sync(c))) return r;
    }
    if (bad) return fail(c, SK_ERANGE, "%s", kRange);
    return SK_OK;
}

int sk_getbit_dev(sk_ctx *c, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets,
                  uint8_t *d_out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    uint64_t mx;
    int r = dev_max_offset(c, n, d_offsets, &mx);
    if (r) return r;
    if (mx >= c->max_bit_offset) return fail(c, SK_ERANGE, "%s", kRange);
    uint32_t id;
    if ((r = str_get(c, key_of(key, len), false, 0, &id))) return r;
    if (id == kNoId) {
        HIPCHK(c, hipMemsetAsync(d_out, 0, n, c->st));
        return sync(c);
    }
    { Prof p_(c, 10);
    HIPCHK(c, sk::launch_getbit_single(c->st, n, d_offsets, c->strs[id].ptr, &c->d_dir[id].len, d_out)); }
    return sync(c);
}

int sk_bitcount(sk_ctx *c, const uint8_t *key, uint64_t len, uint64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t id;
    int r = str_get(c, key_of(key, len), false, 0, &id);
    if (r) return r;
    *out = 0;
    if (id == kNoId) return SK_OK;
    uint64_t l;
    if ((r = str_len(c, id, &l))) return r;
    { Prof p_(c, 11);
    HIPCHK(c, sk::launch_bitcount(c->st, c->strs[id].ptr, l, c->misc.as<uint64_t>())); }
    HIPCHK(c, hipMemcpyAsync(out, c->misc.p, 8, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_strlen(sk_ctx *c, const uint8_t *key, uint64_t len, uint64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    auto it = c->keys.find(key_of(key, len));
    *out = 0;
    if (it == c->keys.end()) return SK_OK;
    if (it->second.type == SK_TYPE_HLL) { // STRLEN of a dense HLL string
        *out = SK_HLL_DENSE_SIZE;
        return SK_OK;
    }
    return str_len(c, it->second.id, out);
}

int sk_bitop(sk_ctx *c, int op, const uint8_t *dest, uint64_t dest_len, uint32_t n_src, const uint64_t *src_off,
             const uint8_t *src_bytes, uint64_t *out_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (op < 0 || op > 3) return fail(c, SK_EINVAL, "ERR syntax error");
    if (op == SK_BITOP_NOT && n_src != 1)
        return fail(c, SK_ESYNTAX, "ERR BITOP NOT must be called with a single source key.");
    if (n_src == 0) return fail(c, SK_EINVAL, "ERR wrong number of arguments for 'bitop' command");
    if (n_src > 64) return fail(c, SK_EINVAL, "BITOP supports at most 64 source keys per call");
    std::vector<const uint8_t *> ptrs(n_src);
    std::vector<uint64_t> lens(n_src);
    std::string dkey = key_of(dest, dest_len);
    uint32_t did = kNoId;
    {
        auto it = c->keys.find(dkey);
        if (it != c->keys.end() && it->second.type == SK_TYPE_STRING) did = it->second.id;
    }
    bool dest_is_src = false;
    uint64_t maxlen = 0;
    for (uint32_t i = 0; i < n_src; i++) {
        uint32_t id;
        int r = str_get(c, key_at(src_off, src_bytes, i), false, 0, &id);
        if (r) return r;
        if (id == kNoId) {
            ptrs[i] = c->strs.empty() ? nullptr : nullptr;
            lens[i] = 0;
            continue;
        }
        if (id == did) dest_is_src = true;
        ptrs[i] = c->strs[id].ptr;
        if ((r = str_len(c, id, &lens[i]))) return r;
        maxlen = std::max(maxlen, lens[i]);
    }
    *out_len = maxlen;
    if (maxlen == 0) { // empty result deletes the destination
        bool removed;
        int r = del_key(c, dkey, &removed);
        return r ? r : sync(c);
    }
    for (uint32_t i = 0; i < n_src; i++)
        if (!ptrs[i]) ptrs[i] = reinterpret_cast<const uint8_t *>(c->d_zero); // len 0: never read
    // destination buffer: in place when dest is a source with room, else fresh
    uint8_t *dst;
    uint8_t *old_buf = nullptr;
    int r = SK_OK;
    if (did != kNoId && c->strs[did].cap >= maxlen) {
        // in place: a source that is also the destination is read and written by
        // the same lane at the same chunk; bytes past the new length must read 0
        dst = c->strs[did].ptr;
        uint64_t old_len;
        if (!dest_is_src) {
            if ((r = str_len(c, did, &old_len))) return r;
            if (old_len > maxlen) HIPCHK(c, hipMemsetAsync(dst + maxlen, 0, old_len - maxlen, c->st));
        }
    } else {
        if (hipMalloc(&dst, round16(maxlen)) != hipSuccess) return fail(c, SK_ENOMEM, "cannot allocate BITOP result");
        if (round16(maxlen) > maxlen) HIPCHK(c, hipMemsetAsync(dst + maxlen, 0, round16(maxlen) - maxlen, c->st));
    }
    HIPCHK(c, c->ptrs.ensure(n_src * 16));
    std::vector<uint8_t> blob(n_src * 16);
    std::memcpy(blob.data(), ptrs.data(), n_src * 8);
    std::memcpy(blob.data() + n_src * 8, lens.data(), n_src * 8);
    HIPCHK(c, hipMemcpyAsync(c->ptrs.p, blob.data(), blob.size(), hipMemcpyHostToDevice, c->st));
    { Prof p_(c, 12);
    HIPCHK(c, sk::launch_bitop(c->st, op, n_src, reinterpret_cast<const uint8_t *const *>(c->ptrs.p),
                               reinterpret_cast<const uint64_t *>(c->ptrs.as<uint8_t>() + n_src * 8), maxlen, dst)); }
    if ((r = sync(c))) return r;
    if (did == kNoId) { // create / replace the destination (BITOP overwrites any type)
        bool removed;
        if ((r = del_key(c, dkey, &removed))) return r;
        uint32_t nid;
        if ((r = str_alloc(c, 16, &nid))) return r;
        HIPCHK(c, hipFree(c->strs[nid].ptr));
        c->strs[nid].ptr = dst;
        c->strs[nid].cap = round16(maxlen);
        c->keys[dkey] = KeyEnt{SK_TYPE_STRING, nid};
        did = nid;
    } else if (dst != c->strs[did].ptr) {
        old_buf = c->strs[did].ptr;
        c->strs[did].ptr = dst;
        c->strs[did].cap = round16(maxlen);
    }
    DirEnt w{c->strs[did].ptr, maxlen, c->strs[did].cap};
    if ((r = dir_write(c, did, w))) return r;
    if ((r = sync(c))) return r;
    if (old_buf) HIPCHK(c, hipFree(old_buf));
    return SK_OK;
}

int sk_get(sk_ctx *c, const uint8_t *key, uint64_t len, uint8_t *buf, uint64_t cap, int64_t *out_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    auto it = c->keys.find(key_of(key, len));
    if (it == c->keys.end()) {
        *out_len = -1;
        return SK_OK;
    }
    if (it->second.type == SK_TYPE_HLL) {
        const HllStr *hx = c->hll_exact && it->second.id < c->hstr.size() ? &c->hstr[it->second.id] : nullptr;
        if (hx && hx->sparse) { // the sparse string as redis-server keeps it
            *out_len = int64_t(16 + hx->ops.size());
            if (cap) std::memcpy(buf, hx->hdr, std::min<uint64_t>(cap, 16));
            if (cap > 16) std::memcpy(buf + 16, hx->ops.data(), std::min<uint64_t>(cap - 16, hx->ops.size()));
            return SK_OK;
        }
        // the slab is the dense body itself: header + one copy
        std::vector<uint8_t> s(SK_HLL_DENSE_SIZE, 0);
        std::memcpy(s.data(), "HYLL", 4);
        s[15] = 0x80;
        if (hx) std::memcpy(s.data(), hx->hdr, 16);
        HIPCHK(c, hipMemcpyAsync(s.data() + 16, c->arena + uint64_t(it->second.id) * kSlabBytes, kSlabBytes,
                                 hipMemcpyDeviceToHost, c->st));
        int r = sync(c);
        if (r) return r;
        *out_len = int64_t(s.size());
        if (cap) std::memcpy(buf, s.data(), std::min<uint64_t>(cap, s.size()));
        return SK_OK;
    }
    uint64_t l;
    int r = str_len(c, it->second.id, &l);
    if (r) return r;
    *out_len = int64_t(l);
    uint64_t ncopy = std::min(cap, l);
    if (ncopy) HIPCHK(c, hipMemcpyAsync(buf, c->strs[it->second.id].ptr, ncopy, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_set(sk_ctx *c, const uint8_t *key, uint64_t len, const uint8_t *val, uint64_t val_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::string k = key_of(key, len);
    bool removed;
    int r = del_key(c, k, &removed); // SET overwrites whatever was there
    if (r) return r;
    uint32_t id;
    if ((r = str_get(c, k, true, val_len, &id))) return r;
    if (val_len) HIPCHK(c, hipMemcpyAsync(c->strs[id].ptr, val, val_len, hipMemcpyHostToDevice, c->st));
    if ((r = sync(c))) return r;
    return str_set_len(c, id, val_len);
}

// GET / SET of a bit string with the value in device memory (cross-GPU BITOP: an operand gathered over RCCL
// becomes a local string without a host round trip; a shard's bytes go straight into a send buffer)
int sk_get_dev(sk_ctx *c, const uint8_t *key, uint64_t len, uint8_t *d_buf, uint64_t cap, int64_t *out_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    auto it = c->keys.find(key_of(key, len));
    if (it == c->keys.end()) {
        *out_len = -1;
        return SK_OK;
    }
    if (it->second.type != SK_TYPE_STRING) return fail(c, SK_EWRONGTYPE, "%s", kWrongType);
    uint64_t l;
    int r = str_len(c, it->second.id, &l);
    if (r) return r;
    *out_len = int64_t(l);
    uint64_t ncopy = std::min(cap, l);
    if (ncopy) HIPCHK(c, hipMemcpyAsync(d_buf, c->strs[it->second.id].ptr, ncopy, hipMemcpyDeviceToDevice, c->st));
    return sync(c);
}

int sk_set_dev(sk_ctx *c, const uint8_t *key, uint64_t len, const uint8_t *d_val, uint64_t val_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::string k = key_of(key, len);
    bool removed;
    int r = del_key(c, k, &removed);
    if (r) return r;
    uint32_t id;
    if ((r = str_get(c, k, true, val_len, &id))) return r;
    if (val_len) HIPCHK(c, hipMemcpyAsync(c->strs[id].ptr, d_val, val_len, hipMemcpyDeviceToDevice, c->st));
    if ((r = sync(c))) return r;
    return str_set_len(c, id, val_len);
}

int sk_bitset_length(sk_ctx *c, const uint8_t *key, uint64_t len, int64_t *out) {
    // Lua of M:RedissonBitSet.java:180-192: fromBit = BITPOS key 1 -1 (first set
    // bit of the LAST byte, -1 if none); toBit = 8*(fromBit/8+1) - fromBit%8
    // (Lua float division, floored modulo); scan GETBIT toBit..fromBit downwards,
    // first 1 -> i+1; else fromBit+1.  GETBIT -1 raises the offset error.
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t id;
    int r = str_get(c, key_of(key, len), false, 0, &id);
    if (r) return r;
    uint64_t l = 0;
    uint8_t last = 0, first = 0;
    if (id != kNoId) {
        if ((r = str_len(c, id, &l))) return r;
        if (l) {
            HIPCHK(c, hipMemcpyAsync(&last, c->strs[id].ptr + l - 1, 1, hipMemcpyDeviceToHost, c->st));
            HIPCHK(c, hipMemcpyAsync(&first, c->strs[id].ptr, 1, hipMemcpyDeviceToHost, c->st));
            if ((r = sync(c))) return r;
        }
    }
    if (l == 0 || last == 0) {
        // fromBit = -1 -> toBit = 0: GETBIT 0, then GETBIT -1 -> error
        if (l && (first & 0x80)) {
            *out = 1;
            return SK_OK;
        }
        return fail(c, SK_ERANGE, "ERR Error running script: %s", kRange);
    }
    int ctz = __builtin_ctz(unsigned(last));
    *out = int64_t(8 * (l - 1) + (8 - ctz));
    return SK_OK;
}

int sk_gen_jackson_longs(uint64_t seed, uint64_t n, uint64_t *off, uint8_t *bytes) {
    static const char pre[] = "[\"java.lang.Long\",";
    const uint64_t plen = sizeof(pre) - 1;
    uint64_t st = seed, t = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        char num[24];
        int nl = snprintf(num, sizeof num, "%lld", (long long)(int64_t)z);
        off[i] = t;
        if (bytes) {
            std::memcpy(bytes + t, pre, plen);
            std::memcpy(bytes + t + plen, num, size_t(nl));
            bytes[t + plen + nl] = ']';
        }
        t += plen + uint64_t(nl) + 1;
    }
    off[n] = t;
    return SK_OK;
}

// ================================================================== Bloom
int sk_bloom_try_init(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t expected, double fpp, int *out_ok) {
    std::lock_guard<std::mutex> g(c->mu);
    int64_t m = sk_bloom_optimal_bits(expected, fpp);
    if (m > kBloomMaxSize)
        return fail(c, SK_ETOOBIG, "Bloom filter can't be greater than %lld. But calculated size is %lld",
                    (long long)kBloomMaxSize, (long long)m);
    int32_t k = sk_bloom_optimal_k(expected, m);
    std::string cfg = "{" + key_of(name, len) + "}__config";
    // tryInit sends EVAL (assert no config) + HMSET in one pipeline
    // (M:RedissonBloomFilter.java:231-240): when the assert fails, the HMSET
    // that follows it still runs, so the new parameters replace the config,
    // and tryInit returns false after re-reading it (Q6).
    *out_ok = c->bloom.count(cfg) ? 0 : 1;
    auto prev = c->bloom.find(cfg);
    const uint64_t seq = prev != c->bloom.end() ? prev->second.seq : c->bloom_seq++; // a replaced config keeps it
    c->bloom[cfg] = BloomCfg{m, k, expected, fpp, sk_rdb::bloom_config_fields(m, k, expected, fpp), seq};
    return SK_OK;
}

int sk_bloom_config(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t *size, int32_t *k, int64_t *expected,
                    double *fpp) {
    std::lock_guard<std::mutex> g(c->mu);
    BloomCfg *b;
    int r = bloom_cfg(c, key_of(name, len), &b);
    if (r) return r;
    if (size) *size = b->size;
    if (k) *k = b->k;
    if (expected) *expected = b->expected;
    if (fpp) *fpp = b->fpp;
    return SK_OK;
}

// shared by the host and device Bloom paths; inputs already on device
static int bloom_add_sorted(sk_ctx *c, uint32_t id, int64_t size, int32_t k, uint64_t n, const uint64_t *d_off,
                            const uint8_t *d_bytes, uint8_t *d_out);

// RBloomFilter.add of n device elements (d_out zeroed here, then 1 for every add that set a bit).  The region
// schedule (sk_kernels.hip "Bloom add, region schedule") in pieces of <= ra_piece() elements, all enqueued without
// a host wait; a hash pass that finds a segment longer than RA_SEGMAX (one element repeated hundreds of times in a
// block) lowers the device word `stop` to its piece number, every apply from that piece on does nothing, and the
// host -- one read at the end -- redoes those pieces on the sort path in order.  k > ra_max_probes() takes the
// sort path whole.
static int bloom_add_device(sk_ctx *c, uint32_t id, int64_t size, int32_t k, uint64_t n, const uint64_t *d_off,
                            const uint8_t *d_bytes, uint8_t *d_out) {
    if (!n) return SK_OK;
    HIPCHK(c, hipMemsetAsync(d_out, 0, n, c->st));
    const uint64_t usize = uint64_t(size);
    if (!(c->bloom_ra_min && n >= c->bloom_ra_min && k >= 1 && uint32_t(k) <= sk::ra_max_probes()))
        return bloom_add_sorted(c, id, size, k, n, d_off, d_bytes, d_out);
    const uint64_t magic = magic_for(usize), piece = sk::ra_piece(k);
    const uint64_t nb = sk::ra_blocks(std::min(n, piece), k), nr = sk::ra_regions(usize);
    HIPCHK(c, c->ra_S.ensure(nb * nr * 4));
    if (sk::rc_seg_interleaved()) HIPCHK(c, c->ra_St.ensure(sk::rc_seg_words(nb, nr) * 4));
    uint32_t *St = sk::rc_seg_interleaved() ? c->ra_St.as<uint32_t>() : c->ra_S.as<uint32_t>();
    HIPCHK(c, c->ra_rec.ensure(nb * sk::ra_chunk_words(k) * 4));
    HIPCHK(c, c->ra_flag.ensure(12)); // [0] the first stopped piece, [1] the one-list slot counter, [2] guard bits
    HIPCHK(c, c->ra_Z.ensure(nb * sk::ra_chunk_words(k) * 4));
    HIPCHK(c, c->ra_GT.ensure(sk::ra_group_table_words(usize) * 8));
    uint32_t *stop = c->ra_flag.as<uint32_t>();
    HIPCHK(c, hipMemsetAsync(stop, 0xff, 4, c->st));
    HIPCHK(c, hipMemsetAsync(stop + 2, 0, 4, c->st));
    uint32_t np = 0;
    for (uint64_t s0 = 0; s0 < n; s0 += piece, np++) {
        const uint64_t m = std::min(piece, n - s0);
        { Prof q_(c, 22);
        HIPCHK(c, sk::launch_bloom_ra_hash(c->st, m, d_off + s0, d_bytes, usize, magic, k, St,
                                           c->ra_rec.as<uint32_t>(), stop, np));
        HIPCHK(c, sk::launch_rc_stranspose(c->st, sk::ra_blocks(m, k), uint32_t(nr), St, c->ra_S.as<uint32_t>())); }
        { Prof q_(c, 23);
        HIPCHK(c, sk::launch_bloom_ra_apply(c->st, m, usize, k, c->ra_S.as<uint32_t>(), c->ra_rec.as<uint32_t>(),
                                            c->strs[id].ptr, c->strs[id].cap, &c->d_dir[id].len, d_out + s0, stop,
                                            np, c->ra_Z.as<uint32_t>(), stop + 1, c->ra_GT.as<uint64_t>())); }
    }
    uint32_t flags[3] = {0, 0, 0};
    HIPCHK(c, hipMemcpyAsync(flags, stop, 12, hipMemcpyDeviceToHost, c->st));
    int r = sync(c);
    if (r) return r;
    if (flags[2]) return fail(c, SK_EDEVICE, "Bloom add apply guard tripped (%u): a broken chain or one-list run", flags[2]);
    const uint32_t first_bad = flags[0];
    for (uint64_t p = first_bad; p < np; p++) { // (first_bad = 0xffffffff: every piece was applied)
        const uint64_t s0 = p * piece, m = std::min(piece, n - s0);
        if ((r = bloom_add_sorted(c, id, size, k, m, d_off + s0, d_bytes, d_out + s0))) return r;
    }
    return SK_OK;
}

// the sort path: d_out already zeroed
static int bloom_add_sorted(sk_ctx *c, uint32_t id, int64_t size, int32_t k, uint64_t n, const uint64_t *d_off,
                            const uint8_t *d_bytes, uint8_t *d_out) {
    // probes per sort: the apply sweeps the touched words of the bit array once per sort, so bigger sorts
    // amortise it (a C3 filter is ~4.2 M lines); keys are idx << 32 | probe number (< 2^32)
    uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t(1) << 27) / uint64_t(k), 0xffffffffull / uint64_t(k)));
    unsigned idx_bits = bits_for(uint64_t(size - 1));
    uint64_t magic = magic_for(uint64_t(size));
    for (uint64_t s = 0; s < n; s += per) {
        uint64_t e = std::min(per, n - s), m = e * uint64_t(k);
        HIPCHK(c, c->keys_a.ensure(m * 8));
        HIPCHK(c, c->keys_b.ensure(m * 8));
        size_t tmp;
        HIPCHK(c, sk::sort_keys_size(m, 32, 32 + idx_bits, &tmp));
        HIPCHK(c, c->sort_tmp.ensure(tmp));
        { Prof p_(c, 6);
        HIPCHK(c, sk::launch_bloom_probes(c->st, e, d_off + s, d_bytes, uint64_t(size), magic, k,
                                          c->keys_a.as<uint64_t>())); }
        { Prof p_(c, 7);
        HIPCHK(c, sk::sort_keys(c->st, c->sort_tmp.p, c->sort_tmp.cap, c->keys_a.as<uint64_t>(),
                                c->keys_b.as<uint64_t>(), m, 32, 32 + idx_bits)); }
        { Prof p_(c, 8);
        HIPCHK(c, sk::launch_bloom_apply(c->st, m, c->keys_b.as<uint64_t>(), c->strs[id].ptr, &c->d_dir[id].len, k,
                                         d_out + s)); }
    }
    return SK_OK;
}

// RBloomFilter.contains of n device elements on stream s (d_out: one reply per element).  Large batches take the
// region schedule (sk_kernels.hip "Bloom contains, region schedule"), in pieces of <= 32 M elements so the probe
// records stay bounded (4 B per probe); small batches and missing filters the one-element-per-thread kernel.
static int bloom_contains_launch(sk_ctx *c, hipStream_t s, uint32_t id, int64_t size, int32_t k, uint64_t n,
                                 const uint64_t *d_off, const uint8_t *d_bytes, uint8_t *d_out) {
    if (!n) return SK_OK;
    const uint64_t usize = uint64_t(size), magic = magic_for(usize);
    const bool region = id != kNoId && c->bloom_rc_min && n >= c->bloom_rc_min && k >= 2 &&
                        uint32_t(k - 1) <= sk::rc_max_probes() && sk::rc_regions(usize) >= 64;
    Prof p_(c, 5, s);
    if (!region) {
        const uint8_t *bits = id == kNoId ? reinterpret_cast<const uint8_t *>(c->d_zero) : c->strs[id].ptr;
        const uint64_t *dl = id == kNoId ? reinterpret_cast<const uint64_t *>(c->d_zero) : &c->d_dir[id].len;
        if (c->bloom_sched == 3) HIPCHK(c, c->bloom_h.ensure(16 * n));
        HIPCHK(c, sk::launch_bloom_contains(s, n, d_off, d_bytes, bits, dl, usize, magic, k, d_out, c->bloom_sched,
                                            c->bloom_h.p));
        return SK_OK;
    }
    const uint64_t piece = uint64_t(32) << 20; // k_bloom_rc_probe serves <= RC_SMAX * RC_TPB blocks
    const uint64_t nb = sk::rc_blocks(std::min(n, piece)), nr = sk::rc_regions(usize);
    HIPCHK(c, c->rc_S.ensure(nb * nr * 4));
    if (sk::rc_seg_interleaved()) HIPCHK(c, c->rc_St.ensure(sk::rc_seg_words(nb, nr) * 4));
    uint32_t *St = sk::rc_seg_interleaved() ? c->rc_St.as<uint32_t>() : c->rc_S.as<uint32_t>();
    HIPCHK(c, c->rc_rec.ensure(nb * sk::rc_chunk_words(k) * 4));
    HIPCHK(c, c->rc_Z.ensure(sk::rc_zero_list_words(usize) * 4));
    HIPCHK(c, c->rc_GT.ensure(sk::rc_group_table_words(usize) * 4));
    for (uint64_t s0 = 0; s0 < n; s0 += piece) {
        uint64_t m = std::min(piece, n - s0);
        { Prof q_(c, 18, s);
        HIPCHK(c, sk::launch_bloom_rc_hash(s, m, d_off + s0, d_bytes, usize, magic, k, St,
                                           c->rc_rec.as<uint32_t>(), d_out + s0));
        if (!sk::rc_probe_reads_st())
            HIPCHK(c, sk::launch_rc_stranspose(s, sk::rc_blocks(m), uint32_t(nr), St, c->rc_S.as<uint32_t>())); }
        { Prof q_(c, 19, s);
        HIPCHK(c, sk::launch_bloom_rc_probe(s, m, usize, k, sk::rc_probe_reads_st() ? St : c->rc_S.as<uint32_t>(),
                                            c->rc_rec.as<uint32_t>(),
                                            c->strs[id].ptr, c->strs[id].cap, d_out + s0, c->rc_Z.as<uint32_t>(),
                                            c->rc_GT.as<uint32_t>())); }
    }
    return SK_OK;
}

static int bloom_prepare(sk_ctx *c, const std::string &nm, int64_t size, int32_t k, bool create, uint32_t *id) {
    BloomCfg *b;
    int r = bloom_cfg(c, nm, &b);
    if (r) return r;
    if (b->size != size || b->k != k) return fail(c, SK_ECONFIG, "%s", kCfgChanged); // addConfigCheck
    if (size <= 0 || k <= 0) return fail(c, SK_EINVAL, "bad Bloom filter config");
    if ((r = str_get(c, nm, create, round16(uint64_t((size + 7) / 8)), id))) return r;
    if (*id != kNoId && (r = str_reserve(c, *id, uint64_t((size + 7) / 8)))) return r;
    return SK_OK;
}

static int stage_elems(sk_ctx *c, uint32_t n, const uint64_t *off, const uint8_t *bytes) {
    uint64_t tot = off[n] - off[0];
    std::vector<uint64_t> o(n + 1);
    for (uint32_t i = 0; i <= n; i++) o[i] = off[i] - off[0];
    HIPCHK(c, c->in_off.ensure((n + 1) * 8ull));
    HIPCHK(c, c->in_bytes.ensure(tot + 16));
    int sr;
    if ((sr = stage_h2d(c, c->in_off.p, o.data(), (n + 1) * 8ull))) return sr;
    if ((sr = stage_h2d(c, c->in_bytes.p, bytes + off[0], tot))) return sr;
    HIPCHK(c, hipMemsetAsync(c->in_bytes.as<uint8_t>() + tot, 0, 16, c->st));
    return sync(c); // o is a host vector
}

// Host ingress in prefix form: element i = prefix ‖ suffix bytes [soff[i], soff[i+1]).  Only the suffixes and u32
// offsets cross the host link (a Jackson Long ships ~21 of its ~39 bytes and 4 instead of 8 offset bytes); the
// elements are rebuilt on the device into in_off / in_bytes (k_expand_prefix).
static int prefix_check(sk_ctx *c, const uint8_t *prefix, uint32_t plen, sk::SkPrefix *pre) {
    if (plen > 255 || (plen && !prefix)) return fail(c, SK_EINVAL, "element prefix of %u bytes (<= 255)", plen);
    std::memset(pre, 0, sizeof *pre);
    if (plen) std::memcpy(pre->w, prefix, plen);
    pre->len = plen;
    return SK_OK;
}
static int stage_prefixed(sk_ctx *c, uint32_t n, const sk::SkPrefix &pre, const uint32_t *soff, const uint8_t *sbytes) {
    const uint64_t tot_s = uint64_t(soff[n] - soff[0]), tot = uint64_t(n) * pre.len + tot_s;
    HIPCHK(c, c->in_soff.ensure((n + 1) * 4ull));
    HIPCHK(c, c->in_sbytes.ensure(tot_s + 16));
    HIPCHK(c, c->in_off.ensure((n + 1) * 8ull));
    HIPCHK(c, c->in_bytes.ensure(tot + 16));
    int sr;
    if ((sr = stage_h2d(c, c->in_soff.p, soff, (n + 1) * 4ull))) return sr;
    if ((sr = stage_h2d(c, c->in_sbytes.p, sbytes + soff[0], tot_s))) return sr;
    HIPCHK(c, sk::launch_expand_prefix(c->st, n, pre, c->in_soff.as<uint32_t>(), c->in_sbytes.as<uint8_t>(),
                                       c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>()));
    HIPCHK(c, hipMemsetAsync(c->in_bytes.as<uint8_t>() + tot, 0, 16, c->st)); // padding contract
    return SK_OK;
}
static uint32_t longest_suffix(uint32_t n, const uint32_t *soff) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; i++) m = std::max(m, soff[i + 1] - soff[i]);
    return m;
}

int sk_pfadd_ids_prefix(sk_ctx *c, uint32_t n, const uint32_t *key_ids, const uint8_t *prefix, uint32_t plen,
                        const uint32_t *soff, const uint8_t *sbytes, uint8_t *out_changed) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!n) return SK_OK;
    sk::SkPrefix pre;
    int r = prefix_check(c, prefix, plen, &pre);
    if (r) return r;
    const uint64_t d = first_dead_handle(c, n, key_ids);
    if (d < n)
        return fail(c, SK_ESTALE,
                    "PFADD: slab id %u is not held by a key (deleted, replaced or never resolved)", key_ids[d]);
    if (plen + uint64_t(longest_suffix(n, soff)) >= sk::long_elem_bytes()) {
        // a long element (addAll's one-element array): the bit-round scan of the full-element path; rebuilt here
        std::vector<uint64_t> off(uint64_t(n) + 1);
        std::vector<uint8_t> bytes;
        bytes.reserve(uint64_t(n) * plen + (soff[n] - soff[0]) + 16);
        for (uint32_t i = 0; i < n; i++) {
            off[i] = bytes.size();
            bytes.insert(bytes.end(), prefix, prefix + plen);
            bytes.insert(bytes.end(), sbytes + soff[i], sbytes + soff[i + 1]);
        }
        off[n] = bytes.size();
        bytes.resize(bytes.size() + 16);
        std::vector<uint32_t> ones(n, 1);
        return pfadd_host_batch(c, n, key_ids, nullptr, ones.data(), off.data(), bytes.data(), out_changed);
    }
    const uint64_t chunk = std::max<uint64_t>(c->max_batch, 1);
    for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
        const uint32_t m = uint32_t(std::min<uint64_t>(chunk, n - c0));
        HIPCHK(c, c->in_ids.ensure(m * 4ull));
        HIPCHK(c, c->out_u8.ensure(m));
        if ((r = stage_h2d(c, c->in_ids.p, key_ids + c0, m * 4ull))) return r;
        if ((r = stage_prefixed(c, m, pre, soff + c0, sbytes))) return r;
        HIPCHK(c, hipMemsetAsync(c->out_u8.p, 0, m, c->st));
        // the same path choice as sk_pfadd_ids for the same batch
        if ((r = pfadd_device(c, m, c->in_ids.as<uint32_t>(), c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>(),
                              nullptr, m, c->out_u8.as<uint8_t>(), pfadd_touched(c, key_ids + c0, m))))
            return r;
        HIPCHK(c, hipMemcpyAsync(out_changed + c0, c->out_u8.p, m, hipMemcpyDeviceToHost, c->st));
        if ((r = sync(c))) return r;
    }
    return SK_OK;
}

int sk_bloom_add_prefix(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                        const uint8_t *prefix, uint32_t plen, const uint32_t *soff, const uint8_t *sbytes,
                        uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    sk::SkPrefix pre;
    int r = prefix_check(c, prefix, plen, &pre);
    if (r) return r;
    uint32_t id;
    if ((r = bloom_prepare(c, key_of(name, len), size, k, true, &id)) || !n) return r;
    if ((r = stage_prefixed(c, n, pre, soff, sbytes))) return r;
    HIPCHK(c, c->out_u8.ensure(n));
    if ((r = bloom_add_device(c, id, size, k, n, c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>(),
                              c->out_u8.as<uint8_t>())))
        return r;
    HIPCHK(c, hipMemcpyAsync(out, c->out_u8.p, n, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_bloom_contains_prefix(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                             const uint8_t *prefix, uint32_t plen, const uint32_t *soff, const uint8_t *sbytes,
                             uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    sk::SkPrefix pre;
    int r = prefix_check(c, prefix, plen, &pre);
    if (r) return r;
    uint32_t id;
    if ((r = bloom_prepare(c, key_of(name, len), size, k, false, &id)) || !n) return r;
    if ((r = stage_prefixed(c, n, pre, soff, sbytes))) return r;
    HIPCHK(c, c->out_u8.ensure(n));
    if ((r = bloom_contains_launch(c, c->st, id, size, k, n, c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>(),
                                   c->out_u8.as<uint8_t>())))
        return r;
    HIPCHK(c, hipMemcpyAsync(out, c->out_u8.p, n, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_bloom_add(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                 const uint64_t *off, const uint8_t *bytes, uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t id;
    int r = bloom_prepare(c, key_of(name, len), size, k, true, &id);
    if (r || !n) return r;
    if ((r = stage_elems(c, n, off, bytes))) return r;
    HIPCHK(c, c->out_u8.ensure(n));
    if ((r = bloom_add_device(c, id, size, k, n, c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>(),
                              c->out_u8.as<uint8_t>())))
        return r;
    HIPCHK(c, hipMemcpyAsync(out, c->out_u8.p, n, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_bloom_contains(sk_ctx *c, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                      const uint64_t *off, const uint8_t *bytes, uint8_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint32_t id;
    int r = bloom_prepare(c, key_of(name, len), size, k, false, &id);
    if (r || !n) return r;
    if ((r = stage_elems(c, n, off, bytes))) return r;
    HIPCHK(c, c->out_u8.ensure(n));
    if ((r = bloom_contains_launch(c, c->st, id, size, k, n, c->in_off.as<uint64_t>(), c->in_bytes.as<uint8_t>(),
                                   c->out_u8.as<uint8_t>())))
        return r;
    HIPCHK(c, hipMemcpyAsync(out, c->out_u8.p, n, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}

int sk_bloom_add_dev(sk_ctx *c, const uint8_t *name, uint64_t len, uint64_t n, const uint64_t *d_off,
                     const uint8_t *d_bytes, uint64_t bytes_len, uint8_t *d_out) {
    (void)bytes_len;
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    BloomCfg *b;
    std::string nm = key_of(name, len);
    int r = bloom_cfg(c, nm, &b);
    if (r) return r;
    uint32_t id;
    if ((r = bloom_prepare(c, nm, b->size, b->k, true, &id))) return r;
    if ((r = bloom_add_device(c, id, b->size, b->k, n, d_off, d_bytes, d_out))) return r;
    return c->async_dev ? SK_OK : sync(c);
}

int sk_bloom_contains_dev(sk_ctx *c, const uint8_t *name, uint64_t len, uint64_t n, const uint64_t *d_off,
                          const uint8_t *d_bytes, uint64_t bytes_len, uint8_t *d_out) {
    (void)bytes_len;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device)); // reads the bit array only: no PFADD settle needed
    BloomCfg *b;
    std::string nm = key_of(name, len);
    int r = bloom_cfg(c, nm, &b);
    if (r) return r;
    uint32_t id;
    if ((r = bloom_prepare(c, nm, b->size, b->k, false, &id))) return r;
    // async: run on the read stream after every main-stream write of bit strings
    bool rs = c->async_dev && c->read_stream;
    hipStream_t s = rs ? c->st2 : c->st;
    if (rs && c->st_wrote_bits) {
        HIPCHK(c, hipEventRecord(c->ev_w, c->st));
        HIPCHK(c, hipStreamWaitEvent(c->st2, c->ev_w, 0));
        c->st_wrote_bits = false;
    }
    if ((r = bloom_contains_launch(c, s, id, b->size, b->k, n, d_off, d_bytes, d_out))) return r;
    if (rs) {
        HIPCHK(c, hipEventRecord(c->ev_r, c->st2));
        c->rd_pending = true;
        return SK_OK;
    }
    if (c->async_dev) return SK_OK;
    return sync(c);
}

int sk_bloom_count(sk_ctx *c, const uint8_t *name, uint64_t len, int32_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    BloomCfg *b;
    std::string nm = key_of(name, len);
    int r = bloom_cfg(c, nm, &b);
    if (r) return r;
    uint32_t id;
    if ((r = str_get(c, nm, false, 0, &id))) return r;
    uint64_t bc = 0;
    if (id != kNoId) {
        uint64_t l;
        if ((r = str_len(c, id, &l))) return r;
        HIPCHK(c, sk::launch_bitcount(c->st, c->strs[id].ptr, l, c->misc.as<uint64_t>()));
        HIPCHK(c, hipMemcpyAsync(&bc, c->misc.p, 8, hipMemcpyDeviceToHost, c->st));
        if ((r = sync(c))) return r;
    }
    // (int) (-size / ((double) hashIterations) * Math.log(1 - bitcount / ((double) size)))  :197
    double v = double(-b->size) / double(b->k) * std::log(1 - double(bc) / double(b->size));
    int32_t res;
    if (v != v) res = 0;
    else if (v >= 2147483647.0) res = 2147483647;
    else if (v <= -2147483648.0) res = INT32_MIN;
    else res = int32_t(v);
    *out = res;
    return SK_OK;
}

} // extern "C"

// ============================================== device memory, timing, RCCL
extern "C" {

int sk_dev_alloc(sk_ctx *c, uint64_t bytes, void **out) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    *out = nullptr;
    if (hipMalloc(out, std::max<uint64_t>(bytes, 16)) != hipSuccess)
        return fail(c, SK_ENOMEM, "cannot allocate %llu device bytes", (unsigned long long)bytes);
    return SK_OK;
}
int sk_dev_free(sk_ctx *c, void *p) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    HIPCHK(c, hipStreamSynchronize(c->st));
    if (p) HIPCHK(c, hipFree(p));
    return SK_OK;
}
int sk_h2d(sk_ctx *c, void *dst, const void *src, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (n) HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->st));
    return sync(c);
}
int sk_d2h(sk_ctx *c, void *dst, const void *src, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (n) HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->st));
    return sync(c);
}
int sk_d2d(sk_ctx *c, void *dst, const void *src, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (n) HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->st));
    return sync(c);
}
int sk_dev_memset(sk_ctx *c, void *p, int v, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (n) HIPCHK(c, hipMemsetAsync(p, v, n, c->st));
    return sync(c);
}

int sk_timer_record(sk_ctx *c, int slot) {
    std::lock_guard<std::mutex> g(c->mu);
    if (slot < 0 || slot >= 16) return fail(c, SK_EINVAL, "timer slot");
    if (c->rd_pending) { // the timer covers read-stream work too
        HIPCHK(c, hipStreamWaitEvent(c->st, c->ev_r, 0));
        c->rd_pending = false;
    }
    if (!c->timers[slot]) HIPCHK(c, hipEventCreate(&c->timers[slot]));
    HIPCHK(c, hipEventRecord(c->timers[slot], c->st));
    return SK_OK;
}
int sk_timer_elapsed(sk_ctx *c, int a, int b, float *ms) {
    std::lock_guard<std::mutex> g(c->mu);
    if (a < 0 || a >= 16 || b < 0 || b >= 16 || !c->timers[a] || !c->timers[b])
        return fail(c, SK_EINVAL, "timer slot");
    HIPCHK(c, hipEventSynchronize(c->timers[b]));
    HIPCHK(c, hipEventElapsedTime(ms, c->timers[a], c->timers[b]));
    return SK_OK;
}

int sk_hll_exact_strings(sk_ctx *c, int on) {
    std::lock_guard<std::mutex> g(c->mu);
    const bool want = on != 0;
    if (want != c->hll_exact && c->hll_next - c->hll_free.size() - c->hll_retired != 0)
        return fail(c, SK_EINVAL, "HLL string mode can change only while no HLL key exists");
    c->hll_exact = want;
    if (want) c->pfadd_path = 1; // the partition path logs the register rises
    return SK_OK;
}

int sk_set_async(sk_ctx *c, int on) {
    std::lock_guard<std::mutex> g(c->mu);
    c->async_dev = on != 0;
    return SK_OK;
}

// Completion tickets for asynchronous submission: a ticket covers all work
// enqueued on the context so far (main and read streams), so a completion
// thread can finish Netty promises without an event-loop thread ever blocking.
int sk_ticket(sk_ctx *c, uint64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    if (c->pf_pending) { // claim/commit path: its conflict check needs the host first
        int r = pfadd_settle(c);
        if (r) return r;
    }
    hipEvent_t a = ev_get(c), b = ev_get(c);
    HIPCHK(c, hipEventRecord(a, c->st));
    HIPCHK(c, hipEventRecord(b, c->st2));
    uint64_t t = c->next_ticket++;
    c->tickets[t] = {a, b};
    *out = t;
    return SK_OK;
}
int sk_poll(sk_ctx *c, uint64_t ticket, int *done) {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->tickets.find(ticket);
    if (it == c->tickets.end()) return fail(c, SK_EINVAL, "unknown ticket");
    hipError_t ea = hipEventQuery(it->second.first), eb = hipEventQuery(it->second.second);
    if ((ea != hipSuccess && ea != hipErrorNotReady) || (eb != hipSuccess && eb != hipErrorNotReady))
        return fail(c, SK_EDEVICE, "HIP: %s", hipGetErrorString(ea != hipSuccess && ea != hipErrorNotReady ? ea : eb));
    *done = ea == hipSuccess && eb == hipSuccess;
    if (*done) { // a finished ticket is released
        c->ev_pool.push_back(it->second.first);
        c->ev_pool.push_back(it->second.second);
        c->tickets.erase(it);
    }
    return SK_OK;
}
int sk_wait(sk_ctx *c, uint64_t ticket) {
    std::pair<hipEvent_t, hipEvent_t> ev;
    {
        std::lock_guard<std::mutex> g(c->mu);
        auto it = c->tickets.find(ticket);
        if (it == c->tickets.end()) return fail(c, SK_EINVAL, "unknown ticket");
        ev = it->second;
        c->tickets.erase(it);
    }
    // outside the lock: other threads keep submitting while this one waits
    hipError_t ea = hipEventSynchronize(ev.first), eb = hipEventSynchronize(ev.second);
    std::lock_guard<std::mutex> g(c->mu);
    c->ev_pool.push_back(ev.first);
    c->ev_pool.push_back(ev.second);
    if (ea != hipSuccess || eb != hipSuccess)
        return fail(c, SK_EDEVICE, "HIP: %s", hipGetErrorString(ea != hipSuccess ? ea : eb));
    return SK_OK;
}

int sk_prof_enable(sk_ctx *c, int on) {
    std::lock_guard<std::mutex> g(c->mu);
    c->prof = on != 0;
    return SK_OK;
}
int sk_prof_only(sk_ctx *c, const char *phase) {
    std::lock_guard<std::mutex> g(c->mu);
    if (!phase) {
        c->prof_mask = 0xffffffffu;
        return SK_OK;
    }
    uint32_t mask = 0; // a comma-separated list of phases
    for (const char *p = phase; *p;) {
        const char *e = strchr(p, ',');
        size_t len = e ? size_t(e - p) : strlen(p);
        int hit = -1;
        for (int i = 0; i < kNumPhases; i++)
            if (strlen(kPhaseNames[i]) == len && strncmp(p, kPhaseNames[i], len) == 0) hit = i;
        if (hit < 0) return fail(c, SK_EINVAL, "unknown phase");
        mask |= 1u << hit;
        p += len + (e ? 1 : 0);
    }
    if (!mask) return fail(c, SK_EINVAL, "unknown phase");
    c->prof_mask = mask;
    return SK_OK;
}
int sk_prof_reset(sk_ctx *c) {
    std::lock_guard<std::mutex> g(c->mu);
    prof_collect(c);
    for (int i = 0; i < 32; i++) c->prof_ms[i] = 0, c->prof_n[i] = 0;
    return SK_OK;
}
int sk_prof_read(sk_ctx *c, const char *phase, uint64_t *launches, double *total_ms) {
    std::lock_guard<std::mutex> g(c->mu);
    if (!std::strcmp(phase, "pfadd_long_fallback")) { // a count, not a timed phase: calls whose long elements were
        *launches = c->long_fallbacks;                // re-hashed per thread after a look-back wait ran out
        *total_ms = 0;
        return SK_OK;
    }
    prof_collect(c);
    for (int i = 0; i < kNumPhases; i++)
        if (!std::strcmp(phase, kPhaseNames[i])) {
            *launches = c->prof_n[i];
            *total_ms = c->prof_ms[i];
            return SK_OK;
        }
    return fail(c, SK_EINVAL, "unknown phase %s", phase);
}

#define NCCLCHK(c, expr)                                                                                               \
    do {                                                                                                               \
        ncclResult_t r__ = (expr);                                                                                     \
        if (r__ != ncclSuccess) return fail((c), SK_EDEVICE, "RCCL error %s", ncclGetErrorString(r__));                \
    } while (0)

int sk_comm_unique_id(uint8_t *out128) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SK_EDEVICE;
    std::memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return SK_OK;
}
int sk_comm_init(sk_ctx *c, int nranks, int rank, const uint8_t *id128) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    ncclUniqueId id;
    std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    if (c->comm) NCCLCHK(c, ncclCommDestroy(c->comm));
    c->comm = nullptr;
    NCCLCHK(c, ncclCommInitRank(&c->comm, nranks, id, rank));
    c->comm_rank = rank;
    c->comm_size = nranks;
    return SK_OK;
}
// all-to-all with per-peer byte counts (send / recv displacements = prefix sums of the counts): the exchange step
// of the range-sharded RBitSet router (cluster.py ShardedBitSet.set_dev / get_dev).  Peers in one RCCL group;
// the rank's own part is a device copy.
int sk_alltoallv(sk_ctx *c, const void *d_send, const uint64_t *send_bytes, void *d_recv, const uint64_t *recv_bytes) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    if (!c->comm) return fail(c, SK_EINVAL, "sk_comm_init first");
    const int W = c->comm_size, me = c->comm_rank;
    std::vector<uint64_t> so(W + 1, 0), ro(W + 1, 0);
    for (int p = 0; p < W; p++) {
        so[p + 1] = so[p] + send_bytes[p];
        ro[p + 1] = ro[p] + recv_bytes[p];
    }
    if (send_bytes[me] != recv_bytes[me]) return fail(c, SK_EINVAL, "alltoallv: own send and receive sizes differ");
    const uint8_t *sb = static_cast<const uint8_t *>(d_send);
    uint8_t *rb = static_cast<uint8_t *>(d_recv);
    if (send_bytes[me]) HIPCHK(c, hipMemcpyAsync(rb + ro[me], sb + so[me], send_bytes[me], hipMemcpyDeviceToDevice, c->st));
    NCCLCHK(c, ncclGroupStart());
    for (int p = 0; p < W; p++) {
        if (p == me) continue;
        if (send_bytes[p]) NCCLCHK(c, ncclSend(sb + so[p], send_bytes[p], ncclUint8, p, c->comm, c->st));
        if (recv_bytes[p]) NCCLCHK(c, ncclRecv(rb + ro[p], recv_bytes[p], ncclUint8, p, c->comm, c->st));
    }
    NCCLCHK(c, ncclGroupEnd());
    return sync(c);
}
// cross-GPU PFMERGE / countWith: register-wise max of 16384-byte arrays
int sk_allreduce_max_u8(sk_ctx *c, uint8_t *d_buf, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (!c->comm) return fail(c, SK_EINVAL, "sk_comm_init first");
    NCCLCHK(c, ncclAllReduce(d_buf, d_buf, n, ncclUint8, ncclMax, c->comm, c->st));
    return sync(c);
}
// BITCOUNT of a range-sharded bitset
int sk_allreduce_sum_u64(sk_ctx *c, uint64_t *d_buf, uint64_t n) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (!c->comm) return fail(c, SK_EINVAL, "sk_comm_init first");
    NCCLCHK(c, ncclAllReduce(d_buf, d_buf, n, ncclUint64, ncclSum, c->comm, c->st));
    return sync(c);
}
// key-sharded BITOP: gather the remote operands, then a local op
int sk_allgather(sk_ctx *c, const void *d_send, void *d_recv, uint64_t bytes_per_rank) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c); // after outstanding read-stream work (an async contains may still be writing the buffer)
    if (!c->comm) return fail(c, SK_EINVAL, "sk_comm_init first");
    NCCLCHK(c, ncclAllGather(d_send, d_recv, bytes_per_rank, ncclUint8, c->comm, c->st));
    return sync(c);
}

} // extern "C"

extern "C" int sk_gen_jackson_longs_dev(sk_ctx *c, uint64_t seed, const uint64_t *d_idx, uint64_t first, uint64_t n,
                                        uint64_t *d_off, uint8_t *d_bytes) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    size_t tmp;
    HIPCHK(c, sk::gen_jackson_scan_size(n, &tmp));
    HIPCHK(c, c->sort_tmp.ensure(std::max<size_t>(tmp, 16)));
    HIPCHK(c, c->keys_a.ensure(std::max<uint64_t>(n, 1) * 8));
    HIPCHK(c, sk::launch_gen_jackson(c->st, n, seed, d_idx, first, c->keys_a.as<uint64_t>(), c->sort_tmp.p,
                                     c->sort_tmp.cap, d_off, d_bytes));
    return sync(c);
}

// ================================================================== persistence (SURVEY 5 "Checkpoint / resume")
// redis-server's own formats (sk_rdb.h): DUMP / RESTORE payloads, SCAN over the keys, and RDB files (SAVE / load).
namespace {

// GET's bytes of an HLL key (sk_get): the exact-mode sparse string, or the dense encoding (kept header in exact
// mode, else "HYLL" + stale cache).  body: the slab (the dense register body), already on the host.
void hll_string_of(const sk_ctx *c, uint32_t id, const uint8_t *body, std::string &out) {
    const HllStr *hx = c->hll_exact && id < c->hstr.size() ? &c->hstr[id] : nullptr;
    if (hx && hx->sparse) {
        out.assign(reinterpret_cast<const char *>(hx->hdr), 16);
        out.append(reinterpret_cast<const char *>(hx->ops.data()), hx->ops.size());
        return;
    }
    out.assign(SK_HLL_DENSE_SIZE, '\0');
    uint8_t hdr[16] = {'H', 'Y', 'L', 'L', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x80};
    std::memcpy(&out[0], hx ? hx->hdr : hdr, 16);
    std::memcpy(&out[16], body, kSlabBytes);
}

// the value of key k as a DUMP payload (*found = false: no such key)
int key_payload(sk_ctx *c, const std::string &k, std::string &out, bool *found) {
    *found = false;
    auto b = c->bloom.find(k);
    if (b != c->bloom.end()) {
        *found = true;
        out = sk_rdb::dump_hash(b->second.fields);
        return SK_OK;
    }
    auto it = c->keys.find(k);
    if (it == c->keys.end()) return SK_OK;
    *found = true;
    std::string v;
    if (it->second.type == SK_TYPE_HLL) {
        std::vector<uint8_t> body(kSlabBytes);
        HIPCHK(c, hipMemcpyAsync(body.data(), c->arena + uint64_t(it->second.id) * kSlabBytes, kSlabBytes,
                                 hipMemcpyDeviceToHost, c->st));
        int r = sync(c);
        if (r) return r;
        hll_string_of(c, it->second.id, body.data(), v);
    } else {
        uint64_t l;
        int r = str_len(c, it->second.id, &l);
        if (r) return r;
        v.assign(l, '\0');
        if (l) HIPCHK(c, hipMemcpyAsync(&v[0], c->strs[it->second.id].ptr, l, hipMemcpyDeviceToHost, c->st));
        if ((r = sync(c))) return r;
    }
    out = sk_rdb::dump_string(v.data(), v.size());
    return SK_OK;
}

// A restored string that is a Redis HLL is adopted at once when GET would return the same bytes afterwards: in
// exact mode (header and sparse opcodes are kept), or for the dense encoding with a stale cache and no other header
// bytes (what this store's GET writes).  Anything else stays a string until its first HLL command, as after SET.
bool hll_eager(const sk_ctx *c, const std::string &v) {
    const uint8_t *s = reinterpret_cast<const uint8_t *>(v.data());
    if (v.size() < 16 || std::memcmp(s, "HYLL", 4) != 0) return false;
    if (c->hll_exact) return s[4] <= 1;
    if (v.size() != SK_HLL_DENSE_SIZE || s[4] != 0 || s[15] != 0x80) return false;
    for (int i = 5; i < 15; i++)
        if (s[i]) return false;
    return true;
}

bool parse_i64(const std::string &s, int64_t *v) {
    if (s.empty() || s.size() > 20) return false;
    char *e = nullptr;
    errno = 0;
    long long x = std::strtoll(s.c_str(), &e, 10);
    if (errno || *e) return false;
    *v = x;
    return true;
}

// a hash restored into the store: a Bloom filter config (size and hashIterations, M:RedissonBloomFilter.java:
// 213-219; the other fields optional), kept with its fields as given
int bloom_from_fields(sk_ctx *c, const sk_rdb::Fields &f, BloomCfg *out) {
    const std::string *size = nullptr, *hi = nullptr, *ex = nullptr, *fp = nullptr;
    for (auto &kv : f) {
        if (kv.first == "size") size = &kv.second;
        else if (kv.first == "hashIterations") hi = &kv.second;
        else if (kv.first == "expectedInsertions") ex = &kv.second;
        else if (kv.first == "falseProbability") fp = &kv.second;
    }
    int64_t sz, k, e = 0;
    if (!size || !hi || !parse_i64(*size, &sz) || !parse_i64(*hi, &k) || (ex && !parse_i64(*ex, &e)))
        return fail(c, SK_EINVAL,
                    "ERR the sketch store keeps hashes only as Bloom filter configs (integer size and hashIterations)");
    // what tryInit can produce (M:RedissonBloomFilter.java:52,72-74): the probe kernels index bits in 32-bit words
    // (sizes < 2^32), and readConfig's Integer.valueOf refuses a hashIterations past int range (:217)
    if (sz < 1 || sz > kBloomMaxSize || k < 1 || k > INT32_MAX)
        return fail(c, SK_EINVAL, "ERR Bloom filter config out of range: size %lld (1..%lld), hashIterations %lld",
                    (long long)sz, (long long)kBloomMaxSize, (long long)k);
    *out = BloomCfg{sz, int32_t(k), e, fp ? std::strtod(fp->c_str(), nullptr) : 0.0, f, 0};
    return SK_OK;
}

// a staging area of dense HLL bodies adopted in bulk: registers unpacked into their slabs by k_hll_unpack
struct HllBulk {
    std::vector<uint32_t> ids;
    std::vector<uint8_t> bodies; // 12,288 B per key
};
int hll_bulk_flush(sk_ctx *c, HllBulk &b) {
    const uint64_t n = b.ids.size();
    if (!n) return SK_OK;
    HIPCHK(c, c->misc.ensure(n * 4));
    HIPCHK(c, c->partial.ensure(n * 12288));
    HIPCHK(c, hipMemcpyAsync(c->misc.p, b.ids.data(), n * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipMemcpyAsync(c->partial.p, b.bodies.data(), n * 12288, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, sk::launch_hll_unpack(c->st, n, c->misc.as<uint32_t>(), c->partial.as<uint8_t>(), c->arena));
    int r = sync(c);
    b.ids.clear();
    b.bodies.clear();
    return r;
}

// a restored value, everything it needs already allocated, so that RESTORE ... REPLACE / load delete the old key
// only once the new value is certain to go in (redis-server decodes the object before it deletes the old key)
struct Restored {
    int kind = 0; // 1 Bloom config, 2 HLL, 3 string
    BloomCfg b;
    uint32_t id = kNoId;
    std::vector<uint8_t> body; // HLL: its 12,288-B dense body
};
int restore_prepare(sk_ctx *c, sk_rdb::Value &v, Restored &p) {
    if (v.type == sk_rdb::kTypeHash) {
        p.kind = 1;
        return bloom_from_fields(c, v.fields, &p.b);
    }
    if (hll_eager(c, v.bytes)) {
        const uint8_t *s = reinterpret_cast<const uint8_t *>(v.bytes.data());
        const bool dense = s[4] == 0 && v.bytes.size() == SK_HLL_DENSE_SIZE; // any dense body decodes
        std::vector<uint8_t> regs;
        if (!dense) regs.resize(kHllBytes);
        if (dense || hll_decode(s, v.bytes.size(), regs.data()) == SK_OK) {
            p.body.resize(12288);
            if (dense) {
                std::memcpy(p.body.data(), s + 16, 12288);
            } else { // sparse (exact mode): its registers in the dense layout
                std::vector<uint8_t> d(SK_HLL_DENSE_SIZE);
                hll_dense_encode(regs.data(), nullptr, d.data());
                std::memcpy(p.body.data(), d.data() + 16, 12288);
            }
            p.kind = 2;
            return hll_alloc(c, &p.id);
        }
    }
    p.kind = 3;
    return str_alloc(c, v.bytes.size(), &p.id);
}
// undo a prepare whose key could not be installed
void restore_release(sk_ctx *c, Restored &p) {
    if (p.kind == 2 && p.id != kNoId) {
        c->hll_live[p.id] = 0;
        c->hll_free.push_back(p.id);
    } else if (p.kind == 3 && p.id != kNoId) {
        (void)str_free(c, p.id);
    }
    p.kind = 0;
}
// install the prepared value as key k (already absent from the store); HLL bodies go through `bulk`
int restore_commit(sk_ctx *c, const std::string &k, sk_rdb::Value &v, Restored &p, HllBulk &bulk) {
    if (p.kind == 1) {
        p.b.seq = c->bloom_seq++;
        c->bloom[k] = std::move(p.b);
        return SK_OK;
    }
    if (p.kind == 2) {
        c->keys[k] = KeyEnt{SK_TYPE_HLL, p.id};
        if (c->hll_exact) {
            const uint8_t *s = reinterpret_cast<const uint8_t *>(v.bytes.data());
            HllStr &h = c->hstr[p.id];
            std::memcpy(h.hdr, s, 16);
            h.sparse = s[4] == 1;
            if (h.sparse) h.ops.assign(s + 16, s + v.bytes.size());
            else std::vector<uint8_t>().swap(h.ops);
        }
        bulk.bodies.insert(bulk.bodies.end(), p.body.begin(), p.body.end());
        bulk.ids.push_back(p.id);
        return bulk.ids.size() >= 8192 ? hll_bulk_flush(c, bulk) : SK_OK;
    }
    c->keys[k] = KeyEnt{SK_TYPE_STRING, p.id};
    if (!v.bytes.empty())
        HIPCHK(c, hipMemcpyAsync(c->strs[p.id].ptr, v.bytes.data(), v.bytes.size(), hipMemcpyHostToDevice, c->st));
    int r = sync(c);
    if (r) return r;
    return str_set_len(c, p.id, v.bytes.size());
}
// prepare, then delete the old key, then install
int restore_replace(sk_ctx *c, const std::string &k, sk_rdb::Value &v, HllBulk &bulk) {
    Restored p;
    int r = restore_prepare(c, v, p);
    if (r) {
        restore_release(c, p);
        return r;
    }
    bool removed;
    if ((r = del_key(c, k, &removed))) {
        restore_release(c, p);
        return r;
    }
    return restore_commit(c, k, v, p, bulk);
}

} // namespace

extern "C" {

// SCAN: a key's position is a 61-bit hash of its name (FNV-1a), so it does not move when the key changes type (a
// string adopted as an HLL, SET over an HLL) or is replaced; the cursor is "the next position" (+ 1, 0 = start).  A call
// returns up to `count` keys of lowest position at or after it, and never splits keys of one position between calls
// (a 61-bit collision), so every key present for the whole scan is returned once.
static uint64_t scan_pos(const std::string &k) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (unsigned char ch : k) h = (h ^ ch) * 0x100000001b3ull;
    return h >> 3;
}
int sk_scan(sk_ctx *c, uint64_t cursor, uint32_t count, uint64_t *next_cursor, uint32_t *out_n, uint64_t *name_off,
            uint8_t *names, uint64_t names_cap, int32_t *types) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    *out_n = 0;
    *next_cursor = 0;
    name_off[0] = 0;
    if (!count) return SK_OK;
    const uint64_t from = cursor ? cursor - 1 : 0;
    struct Ent {
        uint64_t pos;
        const std::string *name;
        int type;
    };
    std::vector<Ent> all;
    all.reserve(c->keys.size() + c->bloom.size());
    for (auto &kv : c->keys) {
        const uint64_t pos = scan_pos(kv.first);
        if (pos >= from) all.push_back(Ent{pos, &kv.first, kv.second.type});
    }
    for (auto &kv : c->bloom) {
        const uint64_t pos = scan_pos(kv.first);
        if (pos >= from) all.push_back(Ent{pos, &kv.first, SK_TYPE_HASH});
    }
    auto lt = [](const Ent &x, const Ent &y) { return x.pos < y.pos || (x.pos == y.pos && *x.name < *y.name); };
    size_t take = std::min<size_t>(count, all.size());
    std::partial_sort(all.begin(), all.begin() + take, all.end(), lt);
    if (take && take < all.size()) { // a position's keys stay together (a hash collision): the last one's wait
        const uint64_t last = all[take - 1].pos;
        if (std::any_of(all.begin() + take, all.end(), [&](const Ent &e) { return e.pos == last; }))
            while (take > 0 && all[take - 1].pos == last) take--;
        if (!take) return fail(c, SK_EINVAL, "sk_scan: count %u is too small for the keys of one position", count);
    }
    uint64_t used = 0;
    size_t n = 0;
    for (; n < take; n++) {
        const std::string &nm = *all[n].name;
        if (used + nm.size() > names_cap) break;
        std::memcpy(names + used, nm.data(), nm.size());
        used += nm.size();
        name_off[n + 1] = used;
        types[n] = all[n].type;
    }
    // a stop for names_cap must not split one position's keys either
    while (n > 0 && n < take && all[n].pos == all[n - 1].pos) n--;
    if (n == 0 && take) return fail(c, SK_EINVAL, "sk_scan: names_cap %llu is too small for the next keys",
                                    (unsigned long long)names_cap);
    *out_n = uint32_t(n);
    if (n < all.size()) *next_cursor = all[n - 1].pos + 2;
    return SK_OK;
}

int sk_dbsize(sk_ctx *c, uint64_t *out) {
    std::lock_guard<std::mutex> g(c->mu);
    *out = uint64_t(c->keys.size() + c->bloom.size());
    return SK_OK;
}

int sk_dump(sk_ctx *c, const uint8_t *key, uint64_t len, uint8_t *buf, uint64_t cap, int64_t *out_len) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    std::string p;
    bool found;
    int r = key_payload(c, key_of(key, len), p, &found);
    if (r) return r;
    *out_len = found ? int64_t(p.size()) : -1;
    if (found && cap) std::memcpy(buf, p.data(), std::min<uint64_t>(cap, p.size()));
    return SK_OK;
}

int sk_restore(sk_ctx *c, const uint8_t *key, uint64_t len, const uint8_t *payload, uint64_t plen, int replace) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    const std::string k = key_of(key, len);
    sk_rdb::Value v;
    std::string why = sk_rdb::load_payload(payload, plen, v);
    if (!why.empty())
        return fail(c, SK_EPAYLOAD, "ERR %s", why.c_str());
    if (!replace && (c->keys.count(k) || c->bloom.count(k)))
        return fail(c, SK_EBUSYKEY, "BUSYKEY Target key name already exists.");
    HllBulk bulk;
    int r = restore_replace(c, k, v, bulk);
    if (r) return r;
    if ((r = hll_bulk_flush(c, bulk))) return r;
    return sync(c);
}

int sk_save(sk_ctx *c, const char *path, uint32_t n_extra, const uint64_t *extra_off, const uint8_t *extra_bytes,
            uint64_t *out_keys) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    uint64_t nk = 0;
    // the caller's records first checked, so a bad one fails before the file is touched
    std::vector<sk_rdb::Value> extra(n_extra);
    for (uint32_t i = 0; i < n_extra; i++) {
        const uint64_t a = extra_off[2 * i + 1], b = extra_off[2 * i + 2];
        std::string why = sk_rdb::load_payload(extra_bytes + a, b - a, extra[i]);
        if (!why.empty()) return fail(c, SK_EPAYLOAD, "ERR extra record %u: %s", i, why.c_str());
    }
    sk_rdb::FileWriter w;
    if (!w.open(path)) return fail(c, SK_EINVAL, "ERR cannot open %s: %s", path, strerror(errno));
    std::vector<std::pair<uint32_t, const std::string *>> hlls, strs;
    for (auto &kv : c->keys) (kv.second.type == SK_TYPE_HLL ? hlls : strs).emplace_back(kv.second.id, &kv.first);
    std::sort(hlls.begin(), hlls.end());
    std::sort(strs.begin(), strs.end());
    // one pinned host buffer for every device read: HLL bodies in batches, strings in pieces
    constexpr uint64_t kBatch = 4096, kPiece = kBatch * 12288;
    uint8_t *pin = nullptr;
    HIPCHK(c, hipHostMalloc(reinterpret_cast<void **>(&pin), kPiece, hipHostMallocDefault));
    auto done = [&](int rc) {
        (void)hipHostFree(pin);
        return rc;
    };
    int r = SK_OK;
    for (size_t b0 = 0; b0 < hlls.size() && !r; b0 += kBatch) {
        const uint64_t n = std::min<uint64_t>(kBatch, hlls.size() - b0);
        std::vector<uint32_t> ids(n);
        for (uint64_t i = 0; i < n; i++) ids[i] = hlls[b0 + i].first;
        if (c->misc.ensure(n * 4) != hipSuccess || c->partial.ensure(n * 12288) != hipSuccess)
            return done(fail(c, SK_ENOMEM, "cannot allocate SAVE staging"));
        if (hipMemcpyAsync(c->misc.p, ids.data(), n * 4, hipMemcpyHostToDevice, c->st) != hipSuccess ||
            sk::launch_hll_pack(c->st, n, c->misc.as<uint32_t>(), c->arena, c->partial.as<uint8_t>()) != hipSuccess ||
            hipMemcpyAsync(pin, c->partial.p, n * 12288, hipMemcpyDeviceToHost, c->st) != hipSuccess)
            return done(fail(c, SK_EDEVICE, "HIP error during SAVE"));
        if ((r = sync(c))) return done(r);
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t id = ids[i];
            const HllStr *hx = c->hll_exact && id < c->hstr.size() ? &c->hstr[id] : nullptr;
            w.record_head(sk_rdb::kTypeString, *hlls[b0 + i].second);
            std::string h;
            if (hx && hx->sparse) { // the sparse string as GET returns it
                sk_rdb::put_len(h, 16 + hx->ops.size());
                h.append(reinterpret_cast<const char *>(hx->hdr), 16);
                h.append(reinterpret_cast<const char *>(hx->ops.data()), hx->ops.size());
                w.put(h);
            } else {
                sk_rdb::put_len(h, SK_HLL_DENSE_SIZE);
                uint8_t hdr[16] = {'H', 'Y', 'L', 'L', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x80};
                if (hx) std::memcpy(hdr, hx->hdr, 16);
                h.append(reinterpret_cast<const char *>(hdr), 16);
                w.put(h);
                w.put(pin + i * 12288, 12288);
            }
            nk++;
        }
    }
    for (auto &e : strs) {
        uint64_t l;
        if ((r = str_len(c, e.first, &l))) return done(r);
        w.record_head(sk_rdb::kTypeString, *e.second);
        std::string h;
        sk_rdb::put_len(h, l);
        w.put(h);
        for (uint64_t o = 0; o < l; o += kPiece) {
            const uint64_t m = std::min(kPiece, l - o);
            if (hipMemcpyAsync(pin, c->strs[e.first].ptr + o, m, hipMemcpyDeviceToHost, c->st) != hipSuccess)
                return done(fail(c, SK_EDEVICE, "HIP error during SAVE"));
            if ((r = sync(c))) return done(r);
            w.put(pin, m);
        }
        nk++;
    }
    std::vector<const std::string *> cfgs;
    for (auto &kv : c->bloom) cfgs.push_back(&kv.first);
    std::sort(cfgs.begin(), cfgs.end(), [](const std::string *a, const std::string *b) { return *a < *b; });
    for (auto *k : cfgs) {
        const sk_rdb::Fields &f = c->bloom[*k].fields;
        w.record_head(sk_rdb::kTypeHash, *k);
        std::string h;
        sk_rdb::put_len(h, f.size());
        for (auto &kv : f) sk_rdb::put_string(h, kv.first), sk_rdb::put_string(h, kv.second);
        w.put(h);
        nk++;
    }
    for (uint32_t i = 0; i < n_extra; i++) {
        const uint64_t a = extra_off[2 * i], b = extra_off[2 * i + 1];
        const uint8_t *p = extra_bytes + extra_off[2 * i + 1];
        const uint64_t pl = extra_off[2 * i + 2] - extra_off[2 * i + 1];
        w.record_head(p[0], std::string(reinterpret_cast<const char *>(extra_bytes + a), b - a));
        w.put(p + 1, pl - 11); // the value: the payload without its type byte and 10-byte trailer
        nk++;
    }
    if (!w.close()) return done(fail(c, SK_EINVAL, "ERR error writing %s: %s", path, strerror(errno)));
    if (out_keys) *out_keys = nk;
    return done(SK_OK);
}

int sk_load(sk_ctx *c, const char *path, sk_take_fn take, void *user, uint64_t *out_keys) {
    std::lock_guard<std::mutex> g(c->mu);
    ENTER(c);
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return fail(c, SK_EINVAL, "ERR cannot open %s: %s", path, strerror(errno));
    struct stat stt;
    if (fstat(fd, &stt) != 0 || stt.st_size <= 0) {
        ::close(fd);
        return fail(c, SK_EPAYLOAD, "ERR %s is empty or unreadable", path);
    }
    const uint64_t n = uint64_t(stt.st_size);
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return fail(c, SK_ENOMEM, "ERR cannot map %s: %s", path, strerror(errno));
    const uint8_t *img = static_cast<const uint8_t *>(m);
    uint64_t nk = 0;
    HllBulk bulk;
    int rc = SK_OK;
    std::string why = sk_rdb::parse_rdb(img, n, [&](const std::string &key, uint8_t type, sk_rdb::Reader &rd) {
        sk_rdb::Value v;
        std::string w = sk_rdb::load_value(rd, type, v);
        if (!w.empty()) return w;
        nk++;
        if (v.type == sk_rdb::kTypeHash && take) {
            const std::string p = sk_rdb::dump_hash(v.fields);
            const int t = take(user, reinterpret_cast<const uint8_t *>(key.data()), key.size(),
                               reinterpret_cast<const uint8_t *>(p.data()), p.size());
            if (t < 0) return std::string("the caller refused the hash ") + key;
            if (t == 1) return std::string();
        }
        if ((rc = restore_replace(c, key, v, bulk))) return std::string("store error: ") + c->err;
        return std::string();
    });
    if (why.empty() && (rc = hll_bulk_flush(c, bulk))) why = "store error: " + c->err;
    munmap(m, n);
    if (!why.empty()) return rc ? rc : fail(c, SK_EPAYLOAD, "ERR %s: %s", path, why.c_str());
    if (out_keys) *out_keys = nk;
    return sync(c);
}

} // extern "C"
