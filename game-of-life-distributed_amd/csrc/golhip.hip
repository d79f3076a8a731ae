// golhip.hip — the C-ABI of libgolhip.so (include/golhip.h).
//
// Host side of the MI355X engine: owns the device boards, sequences the
// step kernels (gol_kernels.hip) on one HIP stream, exchanges halo rows with
// the neighbouring strips (RCCL ring or peer copies) and serves the side
// channels (alive count, flip list, alive list, snapshots).
//
// What each entry point replaces in the reference (gol/distributor.go):
//   golhip_create / _load_bytes  world allocation + fill          :66-80
//   golhip_step                  the turn loop                    :93-173
//   golhip_flips                 initializeAliveCells             :212-220
//   golhip_alive_count           len(calculateAliveCells) ticker  :283-302
//   golhip_alive_cells           calculateAliveCells (final)      :180, :420-432
//   golhip_snapshot_bytes        final/s/q raster streams         :186-191, :234-238
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <functional>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/golhip.h"
#include "gol_kernels.h"

using golk::kHalo;

namespace {

thread_local std::string g_err;

// Page-locked, device-mapped host buffers from golhip_host_alloc: the flip
// stream writes its entries into them straight from the kernel.
struct HostBuf {
    uintptr_t base;
    size_t bytes;
    void *dev;  // device address of base
};
std::mutex g_host_mu;
std::vector<HostBuf> g_host_bufs;

// Device address of [p, p + bytes) if it lies inside one golhip_host_alloc buffer.
void *mapped_device_ptr(const void *p, size_t bytes) {
    std::lock_guard<std::mutex> g(g_host_mu);
    const uintptr_t a = (uintptr_t)p;
    for (const HostBuf &b : g_host_bufs)
        if (a >= b.base && a + bytes <= b.base + b.bytes) return (char *)b.dev + (a - b.base);
    return nullptr;
}

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_OR_FAIL(expr)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(GOLHIP_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Accumulating form for loops that must finish their cleanup: sets `rc` once.
#define HIP_RC(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess && rc == GOLHIP_OK)                                                \
            rc = fail(GOLHIP_EHIP, "%s: %s", #expr, hipGetErrorString(e_));                     \
    } while (0)

#define NCCL_OR_FAIL(expr)                                                                          \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) return fail(GOLHIP_ERCCL, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

// Turns per launch with an instantiated step kernel (24: one word per lane
// only, as 32; 9: four words per lane only, planned only under a cap of
// exactly 9 (depth_cap); see max_depth_for).
constexpr int kDepths[] = {32, 24, 20, 18, 16, 12, 9, 8, 6, 4, 2, 1};
constexpr int kNumDepths = sizeof(kDepths) / sizeof(kDepths[0]);
// trace buffer: 8 totals + (start, end) per (workgroup < 1024, wave < 64)
constexpr int64_t kTraceWords = 8 + 2 * 1024 * 64;

}  // namespace

struct golhip {
    int W = 0, H = 0, Ww = 0;
    int row0 = 0, rows = 0;  // this handle's rows of the torus
    bool strip = false;      // created by golhip_create_strip
    int device = 0;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;

    uint32_t *buf[2] = {nullptr, nullptr};
    int cur = 0;
    int64_t phys_rows = 0;

    int tb_depth = 20;          // per-launch WPL-2 kernels fuse up to 20, the resident kernel 16
    int rows_per_wave = 0;      // 0 = automatic (per depth, from occupancy)
    int cu_count = 0;           // CUs the launches are planned for (option "cu_count": fewer)
    int dev_cu = 0;             // the device's CUs
    bool fill_skip = true;      // option "fill_skip"
    int last_variant = 1;           // kernel family of the last step launch (golhip_perf kernel_variant)
    int skew = 1;                   // option "skew": skewed band stacks (K1w) for per-launch steps
    int skew_young = 0;             // option "skew_young": band height of waves 4..7, % of waves 0..3's (0: by kernel)
    int skew_hcap = -1;             // option "skew_hcap": rows a stack's bottom band gives up (-1: 3 D / 4)
    int skew_prio = 0;              // option "skew_prio": s_setprio 1 for waves 4..7
    int skew_tx = 0;                // option "skew_tx": tiles per K1w workgroup (0: plan, 1 or 2)
    int skew_half = 0;              // option "skew_half": half-wave tiles (0: when fewer wave-rows, 1: whenever possible, -1: never)
    int lds_bpc[4] = {};               // K1r workgroups per CU by (wpl, 512 / 1024 threads) at lds_bpc_bytes of LDS
    int64_t lds_bpc_bytes[4] = {};
    int lds_bpc_stride[4] = {};
    int skew_bpc[kNumDepths][12] = {};  // K1w workgroups per CU by (depth, wpl, half, pairs) (0: not queried)
    int skew_pairs = 5;             // option "skew_pairs": the pair rule (8 LUTs a word-turn) at depth 18 (depth_cap)
    int64_t pair_launches = 0, pair_turns = 0;
    unsigned *skew_err = nullptr;      // host-mapped spin-bound flag of the K1w kernels
    unsigned *skew_err_dev = nullptr;
    int64_t skew_launches = 0;
    int64_t skew_half_launches = 0;
    int lds_band = -1;              // option "lds_band": resident LDS bands K1r (1 on where it fits, 0 off, -1 auto)
    int lds_depth = 0;              // option "lds_depth": turns per K1r super-step (0: plan)
    int lds_xcd = 1;                // option "lds_xcd": consecutive K1r bands on one XCD
    int lds_waves = 0;              // option "lds_waves": K1r waves per workgroup (8 or 16; 0: plan)
    int lds_wg_cu = 1;              // option "lds_wg_cu": K1r bands (workgroups) per CU (1 or 2)
    int lds_stride = 1;             // option "lds_stride": K1r LDS rows at a compile-time stride where instantiated
    int resident_fault = 0;         // option "resident_fault" (tests): K1r band 0 / K1p workgroup 0 never report
                                    // (their neighbours' bounded waits time out: the restore-and-re-run path)
    int lds_age = 0;                // option "lds_age": K1r run rows of a younger wave rank, % of the older's (0: plan)
    int lds_pre = 2;                // option "lds_pre": K1r interior-first turns while the halos travel
                                    // (profiles/r4pre: 8192^2 31.4 -> 33.9 TCUPS at 2; 1: 33.2, 3: 33.1, 4: 32.3)
    uint32_t *lds_edge = nullptr;   // K1r edge rows (golk::lds_band_edge_words)
    int64_t lds_edge_cap = 0;
    int64_t lds_launches = 0;
    int persistent = -1;        // option "persistent": K1p for long torus runs (1 on, 0 off, -1 auto)
    int wpl_opt = 0;            // option "wpl": words per lane (0 = auto, 1, 2, 4)
    int persist_depth = 0;      // option "persist_depth" (0: tb_depth)
    int persist_waves = 0;      // option "persist_waves": waves per workgroup (0: default)
    int paired_bands = 1;       // option "paired_bands": SIMD mates share two bands from both ends (persistent)
    int dummy_rows = 0;         // option "dummy_rows": halo rows taking the kernels' dummy stores (0: all)
    int persist_wg_tx = 0;      // option "persist_wg_tx": tiles across a persistent workgroup (0: plan)
    int persist_half = 1;       // option "persist_half": a D/2-turn remainder runs as the resident kernel's last super-step
    unsigned long long *d_trace = nullptr;  // option "trace": persistent-kernel diagnostics
    unsigned *d_sync = nullptr; // persistent kernel: [0] error, [1..] progress per workgroup
    unsigned *h_err = nullptr;  // pinned copy of the error word
    bool persist_pending = false;
    int64_t persist_launches = 0;
    // resident-launch guard (torus): the board as it was before the step's
    // resident launch, restored and re-run on the per-launch kernels if that
    // launch times out (its workgroups were not all co-resident)
    uint32_t *backup = nullptr;
    bool guarded = false;
    bool guard_light = false;  // the guarded step is one source-keeping launch: its source is the copy
    // the error word d_sync[0] is sticky over a guarded step: only its first
    // resident launch clears it, so a later launch (steps past resident_max
    // turns, a one-rank ring's rounds) can neither wipe an earlier timeout nor
    // run on a drained board unnoticed (its waits see the word and drain too)
    bool err_clear = true;
    int64_t resident_max = golk::kResidentMaxTurns;  // turns a resident launch takes (test hook "resident_max_turns")
    int64_t persist_fallbacks = 0;
    int64_t persist_timeout_ticks = 100000000ll;  // 1 s at the 100 MHz s_memrealtime clock (option "persist_timeout_us")
    int auto_rpw[kNumDepths] = {};  // cache per depth index
    bool loaded = false;
    int il = 0;                 // word layout of the board: 0 canonical, 2 interleaved pairs, 4 quads (= wpl)
    std::atomic<int64_t> turns{0};

    // side-channel scratch
    unsigned long long *d_scalars = nullptr;  // [0] alive, [1] compaction total, [2] hash
    unsigned long long *h_scalars = nullptr;  // pinned mirror
    int64_t alive_turn = -1;                  // turn whose count sits in d_scalars[0]
    unsigned long long *d_blk = nullptr;
    int64_t blk_cap = 0;
    int32_t *d_xy = nullptr;
    int64_t xy_cap = 0;
    unsigned long long *d_run = nullptr;  // flip streams: running list offsets
    int64_t run_cap = 0;
    // flip stream (K5, golhip_flip_stream / golhip_step_flips)
    unsigned long long *d_ftstatus = nullptr;  // look-back word per block (zeroed once)
    int64_t ftstatus_cap = 0;
    unsigned *d_ftticket = nullptr;            // virtual block ids, one counter per turn
    int64_t ftticket_cap = 0;
    unsigned *d_ftctl = nullptr;               // [0] stop, [1] look-back spin error
    void *d_ev = nullptr;                      // entries of a batch
    int64_t ev_cap_bytes = 0;
    unsigned flip_epoch = 0;
    int flip_debug = 0;  // option "flip_debug" (measurement only: wrong lists)
    int flip_cp_groups = 4;  // K5r copy-block groups (GOLHIP_TUNING=1 GOLHIP_FLIP_CP_GROUPS=n, 1..8)
    int flip_overlap = 2;  // option "flip_overlap": how lists reach golhip_host_alloc memory (flip_stream_locked)
    unsigned *d_ftdone = nullptr;  // K5r: kFtShards done counters a turn
    int64_t ftdone_cap = 0;
    int64_t flip_resident = 0;     // K5r launches (flip_overlap 2)
    bool ft_ticket = false;       // K5 block order by ticket (set after a co-residency failure)
    uint64_t ft_est = 0;          // most entries of one turn in the last batch (launch sizing)
    int64_t flip_fallbacks = 0;
    int64_t flip_launches = 0, flip_entries = 0;
    double flip_ms = 0;
    uint8_t *d_stage = nullptr;  // byte staging for load/snapshot
    int64_t stage_cap = 0;
    bool flips_valid = false;
    int64_t flips_turn = -1;

    // ring
    ncclComm_t comm = nullptr;
    // test hook (golhip_test_ring_init): a ring whose halo exchange runs
    // through a host callback instead of RCCL (two processes on one device)
    golhip_test_transport_fn xport = nullptr;
    void *xport_user = nullptr;
    uint32_t *xport_host = nullptr;  // pinned: send up, send down, recv top, recv bottom
    int64_t xport_cap = 0;           // words per block
    bool ringed() const { return comm || xport; }
    bool force_halo = false;    // option "force_halo": one-rank RCCL ring on a whole board (tests)
    int nranks = 1, rank = 0;
    int ring_rows = 0;          // smallest strip of the ring (every rank plans from it)
    int halo_skip = 0;          // option "halo_skip" (measurement only: no exchange, wrong halos)
    int64_t halo_exchanges = 0;
    double halo_ms = 0;         // exchange time on the engine stream (GOLHIP_FLAG_TIMING)

    // measurement
    std::vector<hipEvent_t> ev_pool;
    struct Timed {
        hipEvent_t e0, e1;
        int kind;  // 0 per-launch step, 1 resident step, 2 flip turn (K5), 3 halo exchange
    };
    std::vector<Timed> ev_pending;
    double step_ms = 0, persist_ms = 0;
    int64_t step_launches = 0, step_turns = 0, halo_bytes = 0;
    int64_t persist_turns = 0;

    std::mutex mu;

    int64_t local_words() const { return (int64_t)rows * Ww; }
    uint32_t *cur_rows() const { return buf[cur] + (int64_t)kHalo * Ww; }
    uint32_t *prev_rows() const { return buf[cur ^ 1] + (int64_t)kHalo * Ww; }
    bool torus() const { return nranks == 1 && rows == H; }
};

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
namespace {

int check(golhip_t h) {
    if (!h) return fail(GOLHIP_EINVAL, "null handle");
    return GOLHIP_OK;
}

int set_dev(golhip_t h) {
    HIP_OR_FAIL(hipSetDevice(h->device));
    return GOLHIP_OK;
}

int ensure_stage(golhip_t h, int64_t bytes) {
    if (h->stage_cap >= bytes) return GOLHIP_OK;
    if (h->d_stage) HIP_OR_FAIL(hipFree(h->d_stage));
    h->d_stage = nullptr;
    h->stage_cap = 0;
    HIP_OR_FAIL(hipMalloc(&h->d_stage, (size_t)bytes));
    h->stage_cap = bytes;
    return GOLHIP_OK;
}

int ensure_blk(golhip_t h, int64_t n) {
    if (h->blk_cap >= n) return GOLHIP_OK;
    if (h->d_blk) HIP_OR_FAIL(hipFree(h->d_blk));
    h->d_blk = nullptr;
    h->blk_cap = 0;
    HIP_OR_FAIL(hipMalloc(&h->d_blk, (size_t)std::max<int64_t>(n, 1) * sizeof(unsigned long long)));
    h->blk_cap = n;
    return GOLHIP_OK;
}

int ensure_xy(golhip_t h, int64_t n) {
    if (h->xy_cap >= n) return GOLHIP_OK;
    if (h->d_xy) HIP_OR_FAIL(hipFree(h->d_xy));
    h->d_xy = nullptr;
    h->xy_cap = 0;
    const int64_t cap = std::max<int64_t>(n, 4096);
    HIP_OR_FAIL(hipMalloc(&h->d_xy, (size_t)cap * 2 * sizeof(int32_t)));
    h->xy_cap = cap;
    return GOLHIP_OK;
}

// Rows per launch chunk for byte staging (<= 64 MiB of bytes).
int64_t stage_rows(golhip_t h) {
    const int64_t per = std::max<int64_t>(1, (64ll << 20) / std::max(1, h->W));
    return std::min<int64_t>(per, h->rows);
}

// Depth 9 (quads only) is never a "largest depth": the resident kernels and
// the other word widths have no 9.
int largest_depth(int64_t want) {
    for (int d : kDepths)
        if (d <= want && d != 9 && d != 18) return d;
    return 1;
}
// Depths a plan capped at exactly them alone takes: 9 (quads) and 18 (the
// pair-rule K1w, option "skew_pairs"); depth_cap.
bool special_depth(int d) { return d == 9 || d == 18; }

// The next run of launches for `left` turns of at most `cap` turns each:
// depth d and how many launches of d come next.  The schedule has the fewest
// launches and, among those, the largest smallest launch, in descending
// order: 100 turns at cap 16 run as 4 x 16 + 3 x 12, not 6 x 16 + 4 (a
// 4-turn launch costs about as much as a 16-turn one on a large board:
// 65536^2 x 100 turns ran at 108 vs 122 TCUPS kernel-only).  Far from the
// end the run is `cap` turns; the last 12-13 caps are planned exactly
// (262144^2 x 100 turns at cap 9: 4 x 9 + 8 x 8, not 8 x 9 + 2 x 8 + 2 x 6,
// which a plan of only the last 3-4 caps found).
struct DepthRun {
    int d;
    int64_t n;
};
DepthRun depth_plan(int cap, int64_t left) {
    const int M = special_depth(cap) ? cap : largest_depth(std::max(1, cap));  // 9: quads, 18: pairs (depth_cap)
    if (left <= 0) return {M, 0};
    const int64_t head = std::max<int64_t>(0, left / M - 12);  // launches of M before the planned tail
    const int t = (int)(left - head * M);                      // < 13 M <= 416
    // best[v] = (launches, -smallest launch) for v turns; pick[v] = first depth
    std::vector<int> nl(t + 1, INT_MAX), mn(t + 1, 0), pick(t + 1, 0);
    nl[0] = 0;
    mn[0] = INT_MAX;
    for (int v = 1; v <= t; ++v)
        for (int d : kDepths) {  // descending: ties keep the larger depth
            if (d > M || d > v || nl[v - d] == INT_MAX || (special_depth(d) && M != d)) continue;
            const int n = nl[v - d] + 1, m = std::min(mn[v - d], d);
            if (n < nl[v] || (n == nl[v] && m > mn[v])) {
                nl[v] = n;
                mn[v] = m;
                pick[v] = d;
            }
        }
    std::vector<int> seq;
    for (int v = t; v > 0; v -= pick[v]) seq.push_back(pick[v]);
    std::sort(seq.begin(), seq.end(), std::greater<int>());
    const int d = head > 0 ? M : seq[0];
    int64_t n = head;
    for (int x : seq) n += (x == d);
    return {d, n};
}

// Rows the launch schedule (depth, exchange depth, words per lane) is derived
// from: in a multi-rank ring every rank must pick the same values, so they
// all use the ring's smallest strip.
int sched_rows(golhip_t h) { return (h->ringed() && h->nranks > 1 && h->ring_rows > 0) ? h->ring_rows : h->rows; }

// Relative rate of a (words per lane, waves per workgroup) choice for the
// persistent torus kernel: stored fraction of the computed tile words x band
// efficiency S / (S + 1.75 D) (pipeline fill, see stream_band) x occupancy /
// VALU slots per word-turn (wpl 1: 9 LUT + 2 half-rate shifts + 2 half-rate
// DPP = 17 slots; wpl 2 interleaved: 9 + 1 + 1 half-rate = 13).  Fitted to
// the round-1c sweeps (profiles/r1c): 16384^2 -> wpl 1 with 8 waves,
// 65536^2 -> wpl 2.
// VALU slots per word-turn: 9 LUTs + 2 half-rate DPP moves and 2 half-rate
// funnel shifts per WPL words (interleaved layouts for WPL 2 and 4).
double slots_per_word(int wpl) { return 9.0 + 8.0 / wpl; }

double plan_rate(golhip_t h, int wpl, int nw, int depth) {
    const int tiles = golk::tb_tiles(h->Ww, wpl);
    const double util = (double)h->Ww / (tiles * 62.0 * wpl);
    const double S = (double)sched_rows(h) * tiles / std::max(1.0, (double)h->cu_count * nw);
    const double occ = nw >= 16 ? 1.0 : 0.95;
    return util * S / (S + 1.75 * depth) * occ / slots_per_word(wpl);
}

int default_depth(golhip_t h, int wpl) { return largest_depth(std::min(h->tb_depth, golk::persist_max_depth(wpl))); }

// Waves per workgroup of the persistent kernel: the option, or the better of
// 16 (4 per SIMD: hides VALU latency) and 8 (taller bands: less fill).
int persist_nw_for(golhip_t h, int depth, int wpl) {
    if (h->persist_waves > 0) return h->persist_waves;
    const int def = golk::persist_waves_for(depth, wpl);
    if (def == 16 && plan_rate(h, wpl, 8, depth) > plan_rate(h, wpl, 16, depth) &&
        golk::persist_blocks_per_cu(depth, wpl, 8) >= 1)  // (depth, wpl, 8) instantiated
        return 8;
    return def;
}

// The resident kernel wins on boards whose two buffers sit in the 256 MB
// MALL (16384^2: 61 vs 58 TCUPS); on larger boards the per-launch kernel is
// as fast or faster and far steadier from box to box (65536^2: 114-116 vs
// 96-120 TCUPS over six boxes, 262144^2: 126 vs 105, profiles/r1f), so
// "auto" keeps K1p for buffers of at most 64 MiB (sched_rows: every rank of
// a ring decides alike, as the choice also fixes the word layout).  A row
// strip runs K1p between two deep-halo exchanges (golhip_step).
constexpr int64_t kPersistAutoMaxBytes = 64ll << 20;
int wpl_per_launch(golhip_t h);
bool skew_fills(golhip_t h);
bool lds_fits(golhip_t h, int wpl, golk::LdsBandArgs *out = nullptr);
bool persist_on(golhip_t h) {
    // a multi-rank ring never runs the resident kernel (try_persist_halo):
    // plan words per lane and halos for the per-launch kernels that do run
    if (h->ringed() && h->nranks > 1) return false;
    if (h->persistent >= 0) return h->persistent != 0;
    // round 3: K1w per launch wherever its stacks fill the CUs (16384^2: 82
    // vs 62 TCUPS); smaller boards keep the resident kernel (8192^2: 27.9
    // vs 21.7 for K1w and 12.8 for the per-launch K1, profiles/r3i)
    if (h->skew && skew_fills(h)) return false;
    return (int64_t)sched_rows(h) * h->Ww * 4 <= kPersistAutoMaxBytes;
}

// Words per lane of the step kernels: 2 (interleaved pair layout) cuts the
// shift work per word but quantises tiles at 124 words and halves the band
// height; the option, or whichever plan_rate prefers.
int wpl_for(golhip_t h) {
    if (h->W % 64 != 0) return 1;
    if (h->wpl_opt == 1 || h->wpl_opt == 2) return h->wpl_opt;
    if (h->wpl_opt == 4) return h->W % 128 == 0 ? 4 : 2;
    if ((!h->torus() && !h->ringed()) || !persist_on(h)) return wpl_per_launch(h);
    if (lds_fits(h, 2)) return 2;  // K1r: pairs (11 slots a word-turn against 15)
    auto best = [&](int wpl) {
        const int d = default_depth(h, wpl);
        const int def = golk::persist_waves_for(d, wpl);
        return std::max(plan_rate(h, wpl, def, d), def == 16 ? plan_rate(h, wpl, 8, d) : 0.0);
    };
    // The model charges WPL 2's halved bands too much fill: at 16384^2 it
    // prefers WPL 1 by 4 %, but WPL 2 (8 waves) measured 61.7 vs 59.0 TCUPS
    // on the same box (profiles/r2p/persist_wpl_16384.txt), so WPL 2 wins
    // unless the model puts it more than 5 % behind.
    return best(2) >= 0.95 * best(1) ? 2 : 1;
}

// Words per lane of the per-launch kernels (the option, else the rate model).
int wpl_per_launch(golhip_t h) {
    if (h->W % 64 != 0) return 1;
    if (h->wpl_opt == 1 || h->wpl_opt == 2) return h->wpl_opt;
    if (h->wpl_opt == 4) return h->W % 128 == 0 ? 4 : 2;
    {
        // per-launch kernels (group strips, large boards): the hardware refills freed wave
        // slots, so band height matters less; stored fraction / slots per word
        // (16384-wide strips: 55.6 vs 51.2 TCUPS for wpl 2 vs 1, profiles/r1e)
        // Four words per lane (interleaved quads, 11 slots) run at most 8
        // turns a launch (226 VGPRs); 8- vs 16-turn launches cost ~10 % per
        // turn (fill, twice the HBM passes).  Measured, four vs two words per
        // lane: 131072^2 127.6 vs 120.1 TCUPS, 262144^2 130.8 vs 122.4,
        // 262144 x 32768 (an 8-GPU strip) 124.6 vs 118.5, but 65536^2 107.1
        // vs 115.1 (9 tiles of 248 words for 2048), profiles/r1k; the model
        // gives 65536^2 +0.5 %, hence the 3 % margin.
        auto rate = [&](int wpl) {
            const double deep = (wpl == 4 && h->tb_depth > golk::max_depth_for(4)) ? 0.9 : 1.0;
            return (double)h->Ww / (golk::tb_tiles(h->Ww, wpl) * 62.0 * wpl) / slots_per_word(wpl) * deep;
        };
        const int two = rate(2) >= rate(1) ? 2 : 1;
        return (h->W % 128 == 0 && rate(4) > 1.03 * rate(two)) ? 4 : two;
    }
}

// The wpl = 2 step kernels run on the interleaved pair layout; every other
// kernel reads canonical words (or is layout-agnostic: popcount, row halos).
// Converts the current board in place when the wanted layout changes.
int set_layout(golhip_t h, int il) {
    if (h->il == il) return GOLHIP_OK;
    if (h->loaded) HIP_OR_FAIL(golk::launch_convert_layout(h->cur_rows(), h->local_words(), h->il, il, h->stream));
    h->il = il;
    return GOLHIP_OK;
}
int want_il(golhip_t h) { return wpl_for(h) >= 2 ? wpl_for(h) : 0; }
// After canonical words were written into the current buffer.
int loaded_canonical(golhip_t h) {
    h->il = 0;
    h->loaded = true;
    return set_layout(h, want_il(h));
}

// Most turns one launch may fuse.  In halo mode the `depth` halo rows must
// all come from one neighbour strip, so depth <= strip rows.
bool skew_dims(golhip_t h, int depth, int wpl, int L, golk::SkewArgs *sk);

int depth_cap(golhip_t h, bool halo) {
    if (h->W % 32 != 0) return 1;  // generic kernel: one turn per launch
    // a strip between exchanges runs the resident kernel (its depths) when on
    const int wpl = wpl_for(h);
    int cap = std::min(h->tb_depth, (halo && persist_on(h)) ? golk::persist_max_depth(wpl) : golk::max_depth_for(wpl));
    if (halo) cap = std::min(cap, sched_rows(h));
    // the pair rule (option "skew_pairs", round 6): K1w at 18 turns a launch
    // (the pair state's VGPR bound at two words per lane): whole tori, and
    // ring strips (every rank decides from the ring's smallest strip; the
    // extended rows of a strip's launches only make the stacks easier to
    // plan).  Bit 1: plans on full-width tiles; bit 4: half-wave tile plans
    // too (16384^2 87.9 vs 86.4 TCUPS at 16 on the 9-LUT stages, profiles/r7c)
    bool pair = false;
    if ((h->skew_pairs & 1) && wpl == 2 && cap >= 18) {
        golk::SkewArgs sk{};
        if (skew_dims(h, 18, 2, halo ? sched_rows(h) : h->rows, &sk) && (!sk.half || (h->skew_pairs & 4))) {
            cap = 18;
            pair = true;
        }
    }
    // other whole tori whose K1w plan takes half-wave tiles (bands of ~2D
    // rows, the launch mostly ramps) fuse 16 turns: 16384^2
    // 86.3-86.5 vs 85.5-85.7 TCUPS at 20 (profiles/r5v; 82.1 vs 81.2 in r4y)
    if (!pair && !halo && wpl == 2 && cap > 16) {
        golk::SkewArgs sk{};
        if (skew_dims(h, 20, 2, h->rows, &sk) && sk.half) cap = 16;
    }
    if (cap == 9 && (wpl != 4 || (halo && persist_on(h)))) cap = 8;  // only per-launch quads have 9
    // quads (bit 2): 8 turns a launch on the pair rule instead of 9 on the 9-LUT stages
    if ((h->skew_pairs & 2) && wpl == 4 && cap >= 8) {
        golk::SkewArgs sk{};
        if (skew_dims(h, 8, 4, halo ? sched_rows(h) : h->rows, &sk) && !sk.half) cap = 8;
    }
    return cap;
}

// K5r (flip_overlap 2): copy blocks of the resident flip-stream launch
constexpr int kFlipStreamCopyBlocks = 128;
constexpr int64_t kFlipStreamMinBlocks = 64;  // (64 K words, e.g. 1448^2)

// How many turns the next launch fuses (depth_plan).
int next_depth(golhip_t h, int64_t remaining, bool halo) { return depth_plan(depth_cap(h, halo), remaining).d; }

// torus mode: the handle holds the whole board and wraps rows itself;
// halo mode: rows outside the strip come from the halo rows.
golk::StepArgs step_args(golhip_t h, unsigned long long *alive, bool halo) {
    golk::StepArgs a{};
    a.src = h->buf[h->cur];
    a.dst = h->buf[h->cur ^ 1];
    a.W = h->W;
    a.Ww = h->Ww;
    a.rows_out = h->rows;
    a.dst_base = kHalo;
    if (!halo) {
        a.in.base = kHalo;
        a.in.wrap = h->H;
        a.in.off = 0;
        a.in.rmax = h->H - 1;
    } else {
        a.in.base = 0;
        a.in.wrap = 0;
        a.in.off = kHalo;
        a.in.rmax = (int)h->phys_rows - 1;
    }
    a.rows_per_wave = h->rows_per_wave;
    a.dummy_rows = h->dummy_rows > 0 ? h->dummy_rows : kHalo;
    a.alive = alive;
    a.count_lo = 0;
    a.count_hi = a.rows_out;
    return a;
}

int depth_index(int d) {
    for (int i = 0; i < kNumDepths; ++i)
        if (kDepths[i] == d) return i;
    return kNumDepths - 1;
}

// Per-launch kernel with paired bands (gol_tb_pair_kernel; needs the fill skip).
bool tb_paired(golhip_t h) { return h->paired_bands && h->fill_skip; }

// Rows per wave for a launch of `depth` turns: the user's value, or the
// automatic choice (wave slots = CUs x resident waves per CU).
int rows_per_wave_for(golhip_t h, int depth) {
    if (h->rows_per_wave > 0) return h->rows_per_wave;
    int &c = h->auto_rpw[depth_index(depth)];
    if (c == 0) {
        const int wpl = wpl_for(h);
        const int slots = h->cu_count * golk::tb_wave_slots_per_cu(depth, wpl, tb_paired(h));
        c = golk::auto_rows_per_wave(h->Ww, h->rows, depth, std::max(slots, 1), h->fill_skip, wpl, tb_paired(h));
    }
    return c;
}

hipEvent_t take_event(golhip_t h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int drain_events(golhip_t h) {
    for (auto &p : h->ev_pending) {
        HIP_OR_FAIL(hipEventSynchronize(p.e1));
        float ms = 0;
        HIP_OR_FAIL(hipEventElapsedTime(&ms, p.e0, p.e1));
        (p.kind == 1 ? h->persist_ms : p.kind == 2 ? h->flip_ms : p.kind == 3 ? h->halo_ms : h->step_ms) += ms;
        h->ev_pool.push_back(p.e0);
        h->ev_pool.push_back(p.e1);
    }
    h->ev_pending.clear();
    return GOLHIP_OK;
}

// Halo plan shared by the RCCL ring and the in-process group.
void plan(int strip_rows, int nranks, int rank, int depth, int Ww, golhip_halo_plan_t *p) {
    p->prev_rank = (rank - 1 + nranks) % nranks;
    p->next_rank = (rank + 1) % nranks;
    p->rows = depth;
    p->send_up_row = kHalo;                               // my first `depth` rows -> prev's bottom halo
    p->recv_bottom_row = kHalo + strip_rows;              // <- next's first rows
    p->send_down_row = kHalo + strip_rows - depth;        // my last rows -> next's top halo
    p->recv_top_row = kHalo - depth;                      // <- prev's last rows
    p->bytes = (int64_t)depth * Ww * 4;
}

// RCCL halo exchange for a launch of `depth` turns on stream `st`.  Posting
// order pairs correctly even when prev == next (2 ranks) or both are this
// rank (one-rank ring, option "force_halo"): on every A->B channel the first
// message is A's top rows (B's bottom halo), the second A's bottom rows.
int exchange_rccl(golhip_t h, int depth, hipStream_t st) {
    if (h->halo_skip) return GOLHIP_OK;  // measurement only (option "halo_skip")
    golhip_halo_plan_t p;
    plan(h->rows, h->nranks, h->rank, depth, h->Ww, &p);
    uint32_t *b = h->buf[h->cur];
    const size_t n = (size_t)depth * h->Ww;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->flags & GOLHIP_FLAG_TIMING) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (!e0 || !e1) return fail(GOLHIP_EHIP, "hipEventCreate failed");
        HIP_OR_FAIL(hipEventRecord(e0, st));
    }
    if (h->xport) {
        // test transport: the two send blocks to pinned memory, the callback
        // trades them for the neighbours', the two receive blocks back
        if ((int64_t)n > h->xport_cap) {
            HIP_OR_FAIL(hipHostFree(h->xport_host));
            h->xport_host = nullptr;
            h->xport_cap = 0;
            HIP_OR_FAIL(hipHostMalloc(&h->xport_host, 4 * n * 4, hipHostMallocDefault));
            h->xport_cap = (int64_t)n;
        }
        uint32_t *hb = h->xport_host;
        const size_t bytes = n * 4;
        HIP_OR_FAIL(hipMemcpyAsync(hb, b + (int64_t)p.send_up_row * h->Ww, bytes, hipMemcpyDeviceToHost, st));
        HIP_OR_FAIL(hipMemcpyAsync(hb + n, b + (int64_t)p.send_down_row * h->Ww, bytes, hipMemcpyDeviceToHost, st));
        HIP_OR_FAIL(hipStreamSynchronize(st));
        if (int r = h->xport(h->xport_user, p.prev_rank, p.next_rank, hb, hb + n, hb + 2 * n, hb + 3 * n,
                             (int64_t)bytes))
            return fail(GOLHIP_ERCCL, "test transport returned %d", r);
        HIP_OR_FAIL(hipMemcpyAsync(b + (int64_t)p.recv_top_row * h->Ww, hb + 2 * n, bytes, hipMemcpyHostToDevice, st));
        HIP_OR_FAIL(hipMemcpyAsync(b + (int64_t)p.recv_bottom_row * h->Ww, hb + 3 * n, bytes, hipMemcpyHostToDevice, st));
        HIP_OR_FAIL(hipStreamSynchronize(st));  // the pinned blocks are reused by the next exchange
    } else {
        NCCL_OR_FAIL(ncclGroupStart());
        NCCL_OR_FAIL(ncclSend(b + (int64_t)p.send_up_row * h->Ww, n, ncclUint32, p.prev_rank, h->comm, st));
        NCCL_OR_FAIL(ncclRecv(b + (int64_t)p.recv_bottom_row * h->Ww, n, ncclUint32, p.next_rank, h->comm, st));
        NCCL_OR_FAIL(ncclSend(b + (int64_t)p.send_down_row * h->Ww, n, ncclUint32, p.next_rank, h->comm, st));
        NCCL_OR_FAIL(ncclRecv(b + (int64_t)p.recv_top_row * h->Ww, n, ncclUint32, p.prev_rank, h->comm, st));
        NCCL_OR_FAIL(ncclGroupEnd());
    }
    if (e1) {
        HIP_OR_FAIL(hipEventRecord(e1, st));
        h->ev_pending.push_back({e0, e1, 3});
    }
    h->halo_bytes += 2 * (int64_t)n * 4;
    h->halo_exchanges++;
    return GOLHIP_OK;
}

// Halo mode: output rows [lo, hi) instead of [0, rows) (the deep-halo
// extension), counting only [0, rows).
void shift_rows(golk::StepArgs &a, int lo, int hi) {
    const int rows = a.rows_out;  // the handle's rows (step_args)
    a.rows_out = hi - lo;
    a.dst_base = kHalo + lo;
    a.in.off = kHalo + lo;
    a.dummy_rows = std::max(1, std::min(a.dummy_rows, kHalo + std::min(lo, 0)));  // rows above the outputs
    a.count_lo = -lo;
    a.count_hi = -lo + rows;
}

// Skewed band stacks (K1w, option "skew"): any per-launch step (whole torus
// or a strip's extended rows) whose depth and words per lane have an
// instance.  One workgroup of 8 waves per stack, sized to fill every CU once:
// as many stacks per tile column as the CUs allow, with bands of at least
// D + 3 rows (any height is exact; shorter bands would mostly wait for the
// band below's exports) and the stack's bottom band `hcap` rows shorter (it
// computes its drain in full).  tx = 2 (stacks of 4
// bands, two tiles a workgroup) when the tile count fits the CUs better.
int skew_bpc(golhip_t h, int depth, int wpl, bool half, bool pr) {
    int &c = h->skew_bpc[depth_index(depth)][(wpl == 4 ? 2 : wpl - 1) + (half ? 3 : 0) + (pr ? 6 : 0)];
    if (c == 0) {
        const int b = golk::skew_blocks_per_cu(depth, wpl, half, pr);
        c = b > 0 ? b : -1;
    }
    return c;
}

// The stack plan of a K1w launch over L rows: tiles, workgroup shape, stacks
// and tile kind (no side effects); false if K1w does not apply.
bool skew_dims(golhip_t h, int depth, int wpl, int L, golk::SkewArgs *sk) {
    // the pair rule: 18 turns at two words per lane (no other kernel runs 18,
    // depth_cap), 8 at four (option "skew_pairs" bit 2)
    const bool pr = depth == 18 || (wpl == 4 && depth == 8 && (h->skew_pairs & 2));
    if (!h->skew || h->W % 32 != 0 || !golk::skew_supported(depth, wpl, false, pr)) return false;
    const int hcap = h->skew_hcap >= 0 ? h->skew_hcap : 3 * depth / 4;
    const int smin = depth + 3;
    // half-wave tiles (30 stored lanes a tile, two tiles a wave, the upper one
    // L / 2 rows down): when they need fewer wave-rows than 62-lane tiles
    // (16384^2: 4.5 vs 5 waves a row), or when forced; L must be even
    const bool half_ok = h->skew_half >= 0 && L % 2 == 0 && golk::skew_supported(depth, wpl, true, pr);
    int best_tx = 0, best_nst = 0, best_half = 0, best_tiles = 0;
    double best = 1e300;
    for (int half = 0; half <= (half_ok ? 1 : 0); ++half) {
        if (!half && half_ok && h->skew_half > 0) continue;  // forced
        const int bpc = skew_bpc(h, depth, wpl, half, pr);
        if (bpc < 1) continue;
        const int tiles = half ? (h->Ww + golk::kHalfTileValid * wpl - 1) / (golk::kHalfTileValid * wpl)
                               : golk::tb_tiles(h->Ww, wpl);
        const int Lh = half ? L / 2 : L;
        for (int tx = 1; tx <= 2; ++tx) {
            if (h->skew_tx && tx != h->skew_tx) continue;
            const int sy = 8 / tx, tcols = (tiles + tx - 1) / tx;
            // stacks of Lh / nst + hcap rows whose bands average at least smin + hcap
            // rows (the bottom band gives up hcap of them)
            const int nst = std::min(h->cu_count * bpc / tcols,
                                     Lh / (sy * (smin + hcap) - hcap));
            if (nst < 1) continue;
            // "skew" 1 (default): only when the stacks fill at least 3/4 of the CUs'
            // workgroup slots (smaller tori run the resident kernel, persist_on);
            // 2: whenever a plan exists (tests)
            if (h->skew == 1 && (int64_t)nst * tcols * 4 < (int64_t)h->cu_count * bpc * 3) continue;
            // a wave's buffer-store range (its band, plus L / 2 rows for half tiles) must stay < 2 GiB
            if (((double)Lh / nst + hcap + (half ? Lh : 0)) * h->Ww * 4 >= 2147483648.0) continue;
            // input rows a wave streams; half tiles pay ~2 % for per-lane row addressing
            const double per_wave = ((double)Lh / nst + hcap) / sy * (half ? 1.02 : 1.0);
            if (per_wave < best * 0.999) {
                best = per_wave;
                best_tx = tx;
                best_nst = nst;
                best_half = half;
                best_tiles = tiles;
            }
        }
    }
    if (!best_tx) return false;
    sk->tiles_x = best_tiles;
    sk->pairs = pr ? 1 : 0;
    sk->tx = best_tx;
    sk->nst = best_nst;
    sk->half = best_half;
    sk->hcap = hcap;
    return true;
}

// Whether K1w would run this handle's whole-launch steps (its stacks fill
// the CUs at the per-launch words per lane and depth); persist_on keeps the
// resident kernel for the tori where it would not.
bool skew_fills(golhip_t h) {
    if (!h->skew || h->W % 32 != 0) return false;
    const int wpl = wpl_per_launch(h);
    int cap = std::min(h->tb_depth, golk::max_depth_for(wpl));
    if (cap == 9 && wpl != 4) cap = 8;
    const int depth = cap == 9 ? 9 : largest_depth(cap);
    golk::SkewArgs sk{};
    return skew_dims(h, depth, wpl, sched_rows(h), &sk);
}

bool skew_plan(golhip_t h, int depth, int wpl, const golk::StepArgs &a, golk::SkewArgs *sk) {
    if (!skew_dims(h, depth, wpl, a.rows_out, sk)) return false;
    if (!h->skew_err) {
        void *p = nullptr, *d = nullptr;
        if (hipHostMalloc(&p, sizeof(unsigned), hipHostMallocMapped) != hipSuccess) return false;
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
            (void)hipHostFree(p);
            return false;
        }
        h->skew_err = static_cast<unsigned *>(p);
        h->skew_err_dev = static_cast<unsigned *>(d);
        *h->skew_err = 0;
    }
    const int sy = 8 / sk->tx;
    // The SIMD arbiter serves the older wave of a SIMD (waves 0..3) first: the
    // younger waves' bands are shorter so both finish together.  Measured
    // (round-3 skew_young sweeps, scripts/sweep_opts.py): two words per lane
    // 66-70 %, quads at depth 9 76-82 %.
    // half-wave-tile plans (16-turn launches of ramp-dominated bands): 60 %
    // (16384^2 87.6 vs 86.4 at 68, 83.7 at 55; profiles/r6b); whole tori on
    // full tiles 70 % (65536^2 128.7 vs 127.5-127.8 at 68, 126.4 at 74;
    // profiles/r6i); ring strips 68 % (their sweep is within its noise, r6d)
    const int young = h->skew_young > 0 ? h->skew_young
                      : wpl == 4             ? 78
                      : sk->half             ? 60
                      : a.in.wrap > 0        ? 70
                                             : 68;
    for (int q = 0; q < 8; ++q) sk->wgt[q] = (q < sy && q * sk->tx >= 4) ? young : 100;
    sk->prio_young = h->skew_prio;
    sk->error = h->skew_err_dev;
    sk->trace = h->d_trace;
    return true;
}

// Launch the step kernel for output rows [lo, hi) of this handle (halos, if
// used, already in place); `alive` (nullable) accumulates their popcount.
// No bookkeeping: see finish_launch.
int launch_rows(golhip_t h, int depth, unsigned long long *alive, bool halo, int lo, int hi) {
    const hipStream_t st = h->stream;
    golk::StepArgs a = step_args(h, alive, halo);
    if (lo != 0 || hi != h->rows) shift_rows(a, lo, hi);
    const int wpl = wpl_for(h);
    if (a.rows_out == h->rows) {
        a.rows_per_wave = rows_per_wave_for(h, depth);
    } else if (h->rows_per_wave > 0) {
        a.rows_per_wave = h->rows_per_wave;
    } else {
        const int slots = h->cu_count * golk::tb_wave_slots_per_cu(depth, wpl, tb_paired(h));
        a.rows_per_wave = golk::auto_rows_per_wave(h->Ww, a.rows_out, depth, std::max(slots, 1), h->fill_skip, wpl,
                                                     tb_paired(h));
    }
    // a wave's buffer-store range (two bands of a paired region) must stay < 2 GiB
    a.rows_per_wave = (int)std::min<int64_t>(a.rows_per_wave, ((1ll << 31) - 1) / (8ll * h->Ww));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->flags & GOLHIP_FLAG_TIMING) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (!e0 || !e1) return fail(GOLHIP_EHIP, "hipEventCreate failed");
        HIP_OR_FAIL(hipEventRecord(e0, st));
    }
    hipError_t e;
    golk::SkewArgs sk{};
    const bool skew = skew_plan(h, depth, wpl, a, &sk);
    if (skew) {
        sk.base = a;
        e = golk::launch_skew(sk, depth, wpl, st);
    } else if (h->W % 32 == 0) {
        e = golk::launch_step_tb(a, depth, st, h->fill_skip, wpl, tb_paired(h));
    } else {
        e = golk::launch_step_generic(a, st);
    }
    h->last_variant = h->W % 32 != 0 ? 0 : skew ? 3 : 1;
    if (e != hipSuccess) return fail(GOLHIP_EHIP, "step launch: %s", hipGetErrorString(e));
    if (e1) {
        HIP_OR_FAIL(hipEventRecord(e1, st));
        h->ev_pending.push_back({e0, e1, 0});
        if (h->ev_pending.size() >= 4096) {
            int rc = drain_events(h);
            if (rc) return rc;
        }
    }
    h->step_launches++;
    h->skew_launches += skew;
    h->skew_half_launches += skew && sk.half;
    if (skew && sk.pairs) {
        h->pair_launches++;
        h->pair_turns += depth;
    }
    return GOLHIP_OK;
}

void finish_launch(golhip_t h, int depth, bool count) {
    h->cur ^= 1;
    h->turns += depth;
    h->step_turns += depth;
    if (count) h->alive_turn = h->turns;
}

// One step launch of `depth` turns (halos already in place).
int launch_depth(golhip_t h, int depth, bool count, bool halo) {
    unsigned long long *alive = nullptr;
    if (count) {
        alive = h->d_scalars;
        HIP_OR_FAIL(hipMemsetAsync(alive, 0, sizeof(unsigned long long), h->stream));
    }
    if (int rc = launch_rows(h, depth, alive, halo, 0, h->rows)) return rc;
    finish_launch(h, depth, count);
    return GOLHIP_OK;
}

// Halo mode with deep halos: one exchange of k * depth rows feeds k launches
// of `depth` turns.  Launch i (0-based) steps rows [-ext, rows + ext) with
// ext = (k - 1 - i) * depth, so it also rebuilds the next launch's halo rows
// from the wider halo (the trapezoid: output row -ext needs input rows
// -ext - depth .. , all inside the k * depth received rows).  The extension
// costs 2 * ext extra rows per launch; it saves k - 1 of every k exchanges.
int halo_launches(int rows, int depth, int64_t run) {
    const int64_t k = std::min<int64_t>({(int64_t)kHalo / depth, run, (int64_t)rows / depth});
    return (int)std::max<int64_t>(1, k);
}

// The next exchange of a halo-mode step: one exchange of k * d rows feeds k
// launches (resident: k super-steps) of d turns.  The one schedule of both
// golhip_step and golhip_halo_schedule (what tests/test_dist_gloo.py replays).
// Per-launch kernels take depth_plan's schedule; between exchanges the
// resident kernel runs full-depth super-steps cheaply and only a remainder
// goes to per-launch kernels, which are slow on strips this small: fewest
// short launches, greedily (1000 = 62 x 16 + 8, not 61 x 16 + 12 + 12).
struct HaloRun {
    int d, k;
};
HaloRun halo_next(int cap, int rows, bool resident, int64_t left) {
    DepthRun run = depth_plan(cap, left);
    if (resident) {
        const int d = largest_depth(std::min<int64_t>(cap, left));
        run = {d, left / d};
    }
    return {run.d, halo_launches(rows, run.d, run.n)};
}

int launch_ext(golhip_t h, int depth, bool count, int ext) {
    unsigned long long *alive = nullptr;
    if (count) {
        alive = h->d_scalars;
        HIP_OR_FAIL(hipMemsetAsync(alive, 0, sizeof(unsigned long long), h->stream));
    }
    if (int rc = launch_rows(h, depth, alive, true, -ext, h->rows + ext)) return rc;
    finish_launch(h, depth, count);
    return GOLHIP_OK;
}

// After any stream sync: a persistent launch that timed out leaves the board
// undefined, so it is reported (loudly) and the persistent path is disabled.
int check_persist(golhip_t h) {
    if (!h->persist_pending) return GOLHIP_OK;
    h->persist_pending = false;
    if (*h->h_err) {
        *h->h_err = 0;
        h->persistent = 0;
        return fail(GOLHIP_EHIP, "persistent step kernel timed out waiting for a neighbour workgroup "
                                 "(not all workgroups resident?); board state is undefined, persistent mode disabled");
    }
    return GOLHIP_OK;
}

// Options whose results are wrong by design (they isolate a cost) need the
// environment's explicit consent: GOLHIP_MEASUREMENT=1.
bool measurement_env() {
    const char *v = getenv("GOLHIP_MEASUREMENT");
    return v && !strcmp(v, "1");
}
// Test hooks (exact results, but they force failure paths: a band that never
// publishes, a reported co-residency failure) need GOLHIP_TEST_HOOKS=1.
bool test_hooks_env() {
    const char *v = getenv("GOLHIP_TEST_HOOKS");
    return v && !strcmp(v, "1");
}
// Result-neutral A/B knobs of the kernel plans: the
// defaults are the plans the sweeps under profiles/ chose, and a product
// caller has no reason to move them, so they need GOLHIP_TUNING=1 (or the
// stronger GOLHIP_MEASUREMENT=1).  The product options without consent are
// wpl, persistent, lds_band, skew, timing, persist_timeout_us, force_halo.
constexpr const char *kTuningKeys[] = {
    "persist_depth", "persist_waves", "dummy_rows", "paired_bands", "persist_half", "persist_wg_tx", "trace",
    "cu_count", "fill_skip", "skew_young", "skew_hcap", "skew_prio", "skew_half", "skew_tx", "lds_depth",
    "lds_waves", "lds_wg_cu", "lds_age", "lds_pre", "lds_stride", "lds_xcd", "flip_overlap", "skew_pairs"};
bool tuning_env() {
    const char *v = getenv("GOLHIP_TUNING");
    return (v && !strcmp(v, "1")) || measurement_env();
}
// The consent-gated options, as golhip_build_info() reports them (the CPU
// suite checks the list against the product contract).
constexpr const char *kConsentInfo =
    " CONSENT_MEASUREMENT=halo_skip,flip_debug:1-3"
    " CONSENT_TEST_HOOKS=resident_fault,resident_max_turns,flip_debug:4,golhip_test_ring_init"
    " CONSENT_TUNING=persist_depth,persist_waves,dummy_rows,paired_bands,persist_half,persist_wg_tx,trace,cu_count,"
    "fill_skip,skew_young,skew_hcap,skew_prio,skew_half,skew_tx,lds_depth,lds_waves,lds_wg_cu,lds_age,lds_pre,"
    "lds_stride,lds_xcd,flip_overlap,skew_pairs"
    " PRODUCT_OPTIONS=wpl,persistent,lds_band,skew,timing,persist_timeout_us,force_halo";

// After the stream has synchronised: the K1w spin-bound flag of the launches
// it ran (reported by the call that ran them, then cleared).
int take_skew_err(golhip_t h) {
    if (h->skew_err && *h->skew_err) {
        *h->skew_err = 0;
        return fail(GOLHIP_EHIP, "skewed-band step kernel: a band waited past its spin bound for the band below "
                                 "(board state is undefined)");
    }
    return GOLHIP_OK;
}

int sync_stream(golhip_t h) {
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    if (int rc = take_skew_err(h)) return rc;
    return check_persist(h);
}

// Test hook "resident_fault": 1 = every resident launch's band / workgroup 0
// never reports, 2 = only the first launch of a guarded step (a transient
// starvation: the step's later launches are healthy and must not hide it).
int resident_fault_now(golhip_t h, bool first) {
    return h->resident_fault == 1 || (h->resident_fault == 2 && first) ? 1 : 0;
}

// One resident launch of J super-steps of `depth` turns over the rows of
// `base` (count: the popcount of its last super-step goes to d_scalars);
// returns false (with *rc == 0) when no workgroup plan fits.
bool persist_launch(golhip_t h, golk::StepArgs base, int64_t J, int depth, int wpl, bool count, int *rc,
                    bool half_last = false) {
    *rc = GOLHIP_OK;
    const int nw = persist_nw_for(h, depth, wpl);
    if (golk::persist_blocks_per_cu(depth, wpl, nw) < 1) return false;
    golk::PersistArgs p{};
    // Unpaired fallback: with two waves per SIMD the older one is served
    // first, so the older half of the waves gets 65 % of the rows.
    const int age_split = nw == 8 ? 65 : 0;
    const bool split = age_split > 0 && age_split < 100;
    if (!golk::plan_persist(h->Ww, base.rows_out, depth, h->cu_count, wpl, nw, &p, h->persist_wg_tx)) return false;
    if (2ll * p.S * h->Ww * 4 >= (1ll << 31)) return false;  // a band's buffer-store range
    // every workgroup must be resident at once (they wait on their neighbours):
    // the grid may not exceed what the occupancy query admits on this device
    if ((int64_t)p.cols * p.wg_y > (int64_t)golk::persist_blocks_per_cu(depth, wpl, nw) * h->cu_count) return false;
    if (h->paired_bands && p.wg_sy >= 2 && p.wg_sy % 2 == 0) {
        // the older and the younger wave of a SIMD stream a shared two-band
        // region from both ends and meet where the arbiter's service put them
        p.paired = 1;
    } else if (split && p.wg_sy >= 2 && p.wg_sy % 2 == 0) {
        // rows of a workgroup stack: age_split % to the band rows of the
        // NW/2 oldest waves (w < NW/2 <=> band row < wg_sy/2)
        const int R = p.wg_sy * p.S, hr = p.wg_sy / 2;
        p.S_old = std::max(1, (int)((int64_t)R * age_split / 100 / hr));
        p.S_young = std::max(1, (R - hr * p.S_old) / (p.wg_sy - hr));
        if (hr * p.S_old >= R) p.S_old = p.S_young = 0;
    }
    p.nw = nw;
    if (!h->d_sync) {
        if (hipMalloc(&h->d_sync, (size_t)(2 * h->dev_cu + 2) * sizeof(unsigned)) != hipSuccess ||
            hipHostMalloc(&h->h_err, sizeof(unsigned), hipHostMallocDefault) != hipSuccess) {
            *rc = fail(GOLHIP_ENOMEM, "persistent sync words");
            return false;
        }
        *h->h_err = 0;
    }
    if (count) {
        hipError_t e = hipMemsetAsync(h->d_scalars, 0, sizeof(unsigned long long), h->stream);
        if (e != hipSuccess) { *rc = fail(GOLHIP_EHIP, "memset: %s", hipGetErrorString(e)); return false; }
    }
    const int e0w = h->err_clear ? 0 : 1;  // the error word is sticky over the guarded step
    h->err_clear = false;
    hipError_t e = hipMemsetAsync(h->d_sync + e0w, 0, (size_t)(h->cu_count + 2 - e0w) * sizeof(unsigned), h->stream);
    const int fault = resident_fault_now(h, e0w == 0);
    p.base = base;
    p.base.alive = count ? h->d_scalars : nullptr;
    p.buf0 = h->buf[0];
    p.buf1 = h->buf[1];
    p.first = h->cur;
    p.J = (int)J;
    p.half_last = half_last ? 1 : 0;
    p.error = h->d_sync;
    p.progress = h->d_sync + 1;
    p.timeout_ticks = h->persist_timeout_ticks;
    p.trace = h->d_trace;
    p.fault = fault;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e == hipSuccess && (h->flags & GOLHIP_FLAG_TIMING)) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (e0 && e1) e = hipEventRecord(e0, h->stream);
    }
    if (e == hipSuccess)
        e = golk::launch_persist(p, depth, wpl, h->stream);
    if (e == hipSuccess && e1) {
        e = hipEventRecord(e1, h->stream);
        h->ev_pending.push_back({e0, e1, 1});
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h->h_err, h->d_sync, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream);
    if (e != hipSuccess) {
        *rc = fail(GOLHIP_EHIP, "persistent launch: %s", hipGetErrorString(e));
        return false;
    }
    h->persist_pending = true;
    if (J & 1) h->cur ^= 1;
    const int64_t turns = J * depth - (half_last ? depth / 2 : 0);
    h->turns += turns;
    h->persist_turns += turns;
    h->persist_launches++;
    if (count) h->alive_turn = h->turns;
    return true;
}

// The resident kernel's depths: 4, 8, 16 and, at one word per lane, 32 (its
// instantiations); the per-launch depths 20, 24, 12, 9, 6 are not among them.
int persist_depth_for(golhip_t h, int wpl) {
    const int cap = std::min(h->persist_depth > 0 ? h->persist_depth : h->tb_depth, golk::persist_max_depth(wpl));
    for (int d : {32, 16, 8, 4})
        if (d <= cap) return d;
    return 1;
}

// Keep the board recoverable before a step's first resident launch: a copy
// of this handle's rows that golhip_step restores (and then re-runs the step
// on the per-launch kernels) if a resident launch times out.  False (rc 0)
// if there is no room for the copy: then no resident launch this step.
// keeps_src: the step is one launch that never writes its source buffer (K1r,
// reads it once into LDS and writes only the other buffer) and nothing runs
// after it, so the source itself is the copy (a timeout leaves it intact).
bool take_guard(golhip_t h, int *rc, bool keeps_src = false) {
    *rc = GOLHIP_OK;
    if (h->guarded) return true;  // a step of several resident launches keeps its first copy
    h->err_clear = true;          // the step's first resident launch clears the error word
    if (keeps_src) {
        h->guarded = true;
        h->guard_light = true;
        return true;
    }
    const size_t bytes = (size_t)h->local_words() * 4;
    if (!h->backup && hipMalloc(&h->backup, bytes) != hipSuccess) {
        h->backup = nullptr;
        return false;
    }
    hipError_t e = hipMemcpyAsync(h->backup, h->cur_rows(), bytes, hipMemcpyDeviceToDevice, h->stream);
    if (e != hipSuccess) {
        *rc = fail(GOLHIP_EHIP, "resident-launch guard copy: %s", hipGetErrorString(e));
        return false;
    }
    h->guarded = true;
    return true;
}

// The K1r plan of this torus at `wpl` words per lane (no side effects):
// one band per CU of at least D rows, both LDS buffers of a band in one
// workgroup's LDS, every workgroup resident.  Depth: the option, else 12
// (profiles/r4k-r4n sweeps: 8192^2 31.8 TCUPS at 12 vs 31.7 at 8 and 30.6 at
// 16; 5120^2 17.9 vs 17.0 and 17.7; 4096^2 13.4 vs 13.0 and 13.6), at most
// the row count.  False if K1r does not apply.
bool lds_fits(golhip_t h, int wpl, golk::LdsBandArgs *out) {
    if (h->lds_band == 0 || !h->torus() || h->W % 128 != 0 || (wpl == 2 && h->W % 64 != 0)) return false;
    if (h->nranks > 1) return false;
    // waves: 16 where a row's pairs fill whole waves at least twice and the
    // 1024 threads exactly (8192 wide: 40.9 vs 39.4 TCUPS at depth 10; 5120 /
    // 4096 wide lose a quarter with 16, their runs too short; 12288 wide, 960
    // of 1024 threads busy: 12.0 against K1p's 13.0 at 12288 x 2048;
    // profiles/r5m, r5n), else 8; depth 10 at 16 waves, else 12 (r5m: 8192^2
    // at 8 waves 39.8 / 39.4 / 38.9 at 10 / 12 / 14, 5120^2 21.2 / 21.6 / 21.2)
    const int P2 = h->Ww / 2;
    const int waves = h->lds_waves > 0 ? h->lds_waves
                      : (wpl == 2 && P2 % 64 == 0 && P2 >= 128 && 1024 % P2 == 0) ? 16 : 8;
    const int D = h->lds_depth > 0 ? h->lds_depth : std::min(waves == 16 ? 10 : 12, h->rows);
    if (h->rows < D || D < 1) return false;
    const int nt = 64 * waves;
    // auto: only where the rows' pairs (words) keep >= 90 % of the threads busy
    // (runs of whole columns: 512 / P runs each; 12288 x 2048 = 192 pairs a row
    // keeps 384 of 512 and ran 11.0 vs K1p's 13.0 TCUPS, while 1024^2 .. 8192^2,
    // 3072^2 and 8192 x 4096 run 1.3-2.1x K1p, profiles/r4x)
    if (h->lds_band < 0) {
        const int64_t P = h->Ww / wpl, units = P * std::max<int64_t>(1, nt / P);
        const int64_t slots = (units + nt - 1) / nt * nt;  // passes x threads
        if (10 * units < 9 * slots) return false;
    }
    // one progress word per band after d_sync's error word (2 dev_cu + 2 words)
    const int nb = std::min(std::min(h->cu_count, h->dev_cu) * h->lds_wg_cu, h->rows / D);
    if (nb < 1) return false;
    const int hmax = (h->rows + nb - 1) / nb;
    // the row stride: pairs always the two-plane row (Ww + 8, gol_kernels.hip K1r)
    const int stride = golk::lds_band_stride(h->Ww, wpl, nt);
    const int64_t bytes = golk::lds_band_lds_bytes(hmax, D, stride);
    if (bytes > 160 * 1024 - 256) return false;  // (the kernel's few static LDS bytes)
    const int slot = (wpl == 2 ? 1 : 0) + (nt == 1024 ? 2 : 0);
    int &bpc = h->lds_bpc[slot];
    if (bpc == 0 || h->lds_bpc_bytes[slot] != bytes || h->lds_bpc_stride[slot] != stride) {
        bpc = std::max(0, golk::lds_band_blocks_per_cu(wpl, nt, stride, bytes));
        h->lds_bpc_bytes[slot] = bytes;
        h->lds_bpc_stride[slot] = stride;
    }
    if ((int64_t)nb > (int64_t)bpc * h->cu_count) return false;
    if (out) {
        out->Ww = h->Ww;
        out->rows = h->rows;
        out->nb = nb;
        out->D = D;
        out->hmax = hmax;
        out->xcd = h->lds_xcd;
        out->nt = nt;
        out->stride = stride;
        out->rt_stride = h->lds_stride ? 0 : 1;
        out->fault = h->resident_fault != 0;
        out->pre = h->lds_pre;
        // the SIMD arbiter's age order, where whole waves share a run (a row's
        // pairs a multiple of 64): 16 waves (4 ranks) 60 %, 8 waves 70 %
        // (profiles/r5z: 8192^2 40.2 -> 43.8 TCUPS, 4096^2 17.1 -> 17.8); runs
        // that straddle waves stay equal (5120^2 +1 % at 80, 2048^2 -5 %)
        const bool whole = wpl == 2 && P2 % 64 == 0;
        out->age = h->lds_age > 0 ? h->lds_age : !whole ? 100 : waves == 16 ? 60 : 70;
    }
    return true;
}

// Torus: all `left` turns as one K1r launch (under the step guard, like
// K1p); returns the turns run (0 if K1r does not apply).
int64_t try_lds(golhip_t h, int64_t left, bool count_last, int *rc) {
    *rc = GOLHIP_OK;
    if (left < 2 || !(h->il == 0 || h->il == 2)) return 0;
    const int64_t run = golk::resident_turns(left, h->resident_max);  // 32-bit super-step arithmetic in the kernel
    const int wpl = h->il == 2 ? 2 : 1;
    golk::LdsBandArgs p{};
    if (!lds_fits(h, wpl, &p)) return 0;
    const int64_t ew = golk::lds_band_edge_words(p.nb, p.D, p.stride);
    if (ew > h->lds_edge_cap) {
        if (hipFree(h->lds_edge) != hipSuccess) {
            *rc = fail(GOLHIP_EHIP, "hipFree (K1r edges)");
            return 0;
        }
        h->lds_edge = nullptr;
        h->lds_edge_cap = 0;
        if (hipMalloc(&h->lds_edge, (size_t)ew * 4) != hipSuccess) {
            h->lds_edge = nullptr;
            return 0;
        }
        h->lds_edge_cap = ew;
    }
    if (!h->d_sync) {
        if (hipMalloc(&h->d_sync, (size_t)(2 * h->dev_cu + 2) * sizeof(unsigned)) != hipSuccess ||
            hipHostMalloc(&h->h_err, sizeof(unsigned), hipHostMallocDefault) != hipSuccess) {
            *rc = fail(GOLHIP_ENOMEM, "resident sync words");
            return 0;
        }
        *h->h_err = 0;
    }
    if (!take_guard(h, rc, count_last && run == left)) return 0;
    const bool count = count_last && run == left;
    hipError_t e = count ? hipMemsetAsync(h->d_scalars, 0, sizeof(unsigned long long), h->stream) : hipSuccess;
    const int e0w = h->err_clear ? 0 : 1;  // the error word is sticky over the guarded step
    h->err_clear = false;
    if (e == hipSuccess) e = hipMemsetAsync(h->d_sync + e0w, 0, (size_t)(p.nb + 1 - e0w) * sizeof(unsigned), h->stream);
    p.fault = resident_fault_now(h, e0w == 0);
    p.src = h->cur_rows();
    p.dst = h->prev_rows();
    p.edge = h->lds_edge;
    p.error = h->d_sync;
    p.progress = h->d_sync + 1;
    p.alive = count ? h->d_scalars : nullptr;
    p.timeout_ticks = h->persist_timeout_ticks;
    p.turns = (int)run;
    p.trace = h->d_trace;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (e == hipSuccess && (h->flags & GOLHIP_FLAG_TIMING)) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (e0 && e1) e = hipEventRecord(e0, h->stream);
    }
    if (e == hipSuccess) e = golk::launch_lds_band(p, wpl, h->stream);
    if (e == hipSuccess && e1) {
        e = hipEventRecord(e1, h->stream);
        h->ev_pending.push_back({e0, e1, 1});
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h->h_err, h->d_sync, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream);
    if (e != hipSuccess) {
        *rc = fail(GOLHIP_EHIP, "resident LDS-band launch: %s", hipGetErrorString(e));
        return 0;
    }
    h->persist_pending = true;
    h->cur ^= 1;
    h->last_variant = 4;
    h->turns += run;
    h->persist_turns += run;
    h->persist_launches++;
    h->lds_launches++;
    if (count) h->alive_turn = h->turns;
    return run;
}

// Torus: J super-steps of `depth` turns in one resident launch; returns the
// turns run (0 if the persistent path does not apply).
int64_t try_persist(golhip_t h, int64_t left, bool count_last, int *rc) {
    *rc = GOLHIP_OK;
    if (!persist_on(h) || h->W % 32 != 0 || !h->torus()) return 0;
    if (int64_t n = try_lds(h, left, count_last, rc)) return n;
    if (*rc) return 0;
    const int wpl = wpl_for(h);
    const int depth = persist_depth_for(h, wpl);
    if (depth < 4 || golk::persist_blocks_per_cu(depth, wpl, persist_nw_for(h, depth, wpl)) < 1) return 0;
    int64_t J = golk::resident_turns(left, h->resident_max) / depth;  // (32-bit super-step counts in the kernel)
    if (J < 2) return 0;
    // a remainder of exactly depth / 2 turns (1000 = 62 x 16 + 8) becomes a
    // last, half-depth super-step
    const bool half = h->persist_half && left - J * depth == depth / 2;
    if (half) ++J;
    const int64_t turns = J * depth - (half ? depth / 2 : 0);
    const bool count = count_last && turns == left;
    if (!take_guard(h, rc)) return 0;
    if (!persist_launch(h, step_args(h, nullptr, false), J, depth, wpl, count, rc, half)) {
        h->guarded = false;  // nothing resident ran: no check needed
        return 0;
    }
    return turns;
}

// Row strip between two deep-halo exchanges of k * d rows: the k launches of
// d turns as one resident launch of k super-steps over the rows
// [-(k-1) d, rows + (k-1) d) (the outer rows go stale one super-step at a
// time, as in the per-launch trapezoid, and are never read by a kept row).
// Only in the one-rank ring (force_halo), under the guard step_locked took
// at the start of the step: a timeout restores the board and re-runs the
// step on per-launch kernels, exchanges included, which is safe with no
// other rank.  Never in a multi-rank ring: a re-run on one rank alone would
// desynchronise the ring, so ring strips stay on per-launch kernels (K1w).
bool try_persist_halo(golhip_t h, int d, int k, bool count, int *rc) {
    *rc = GOLHIP_OK;
    if (!persist_on(h) || h->W % 32 != 0 || k < 2 || d < 4) return false;
    if ((h->ringed() && h->nranks > 1) || !h->guarded) return false;
    const int wpl = wpl_for(h);
    if (d != persist_depth_for(h, wpl)) return false;
    const int e = (k - 1) * d;
    golk::StepArgs a = step_args(h, nullptr, true);
    shift_rows(a, -e, h->rows + e);
    return persist_launch(h, a, k, d, wpl, count, rc);
}

int start_flips(golhip_t h) {
    const int64_t nw = h->local_words();
    const int64_t nb = golk::compact_blocks(nw);
    int rc = ensure_blk(h, nb);
    if (rc) return rc;
    HIP_OR_FAIL(golk::launch_compact_count(h->cur_rows(), h->prev_rows(), nw, h->d_blk, h->stream));
    HIP_OR_FAIL(golk::launch_compact_scan(h->d_blk, nb, h->d_scalars + 1, h->stream));
    h->flips_valid = true;
    h->flips_turn = h->turns;
    return GOLHIP_OK;
}

// Finish a compaction started with count+scan: read the total, scatter, copy out.
int finish_compact(golhip_t h, const uint32_t *a, const uint32_t *b, int32_t *xy, uint64_t cap, uint64_t *n) {
    HIP_OR_FAIL(hipMemcpyAsync(h->h_scalars + 1, h->d_scalars + 1, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    const uint64_t total = h->h_scalars[1];
    if (n) *n = total;
    if (total > cap || (!xy && total > 0))
        return fail(GOLHIP_ERANGE, "buffer holds %llu cells, %llu needed", (unsigned long long)cap,
                    (unsigned long long)total);
    if (total == 0) return GOLHIP_OK;
    int rc = ensure_xy(h, (int64_t)total);
    if (rc) return rc;
    HIP_OR_FAIL(golk::launch_compact_scatter(a, b, h->local_words(), h->Ww, h->row0, h->d_blk, h->d_xy, h->il, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(xy, h->d_xy, total * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    return GOLHIP_OK;
}

int create_common(int32_t width, int32_t height, int32_t row0, int32_t rows, int32_t device, uint32_t flags,
                  bool strip, golhip_t *out) {
    if (!out) return fail(GOLHIP_EINVAL, "out is null");
    *out = nullptr;
    if (width <= 0 || height <= 0) return fail(GOLHIP_EINVAL, "bad board %dx%d", width, height);
    if (rows <= 0 || row0 < 0 || (int64_t)row0 + rows > height)
        return fail(GOLHIP_EINVAL, "bad strip rows [%d, %d) of %d", row0, row0 + rows, height);
    int ndev = 0;
    HIP_OR_FAIL(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(GOLHIP_EINVAL, "device %d of %d", device, ndev);
    HIP_OR_FAIL(hipSetDevice(device));
    golhip *h = new golhip();
    h->W = width;
    h->H = height;
    h->Ww = (width + 31) / 32;
    h->row0 = row0;
    h->rows = rows;
    h->strip = strip;
    h->device = device;
    h->flags = flags;
    h->phys_rows = (int64_t)rows + 2 * kHalo;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->cu_count = prop.multiProcessorCount;
        if (h->cu_count <= 0) h->cu_count = 256;
        h->dev_cu = h->cu_count;
    }
    const size_t bytes = (size_t)h->phys_rows * h->Ww * sizeof(uint32_t);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) h->own_stream = true;
    if (e == hipSuccess) e = hipMalloc(&h->buf[0], bytes);
    if (e == hipSuccess) e = hipMalloc(&h->buf[1], bytes);
    // zeroed on the handle's own stream: it is non-blocking, so a plain
    // hipMemset (null stream, asynchronous for device memory) could still be
    // running when the first load / fill_random on `stream` writes the board
    if (e == hipSuccess) e = hipMemsetAsync(h->buf[0], 0, bytes, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(h->buf[1], 0, bytes, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMalloc(&h->d_scalars, 4 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipHostMalloc(&h->h_scalars, 4 * sizeof(unsigned long long), hipHostMallocDefault);
    if (e != hipSuccess) {
        int code = (e == hipErrorOutOfMemory) ? GOLHIP_ENOMEM : GOLHIP_EHIP;
        fail(code, "allocating %zu bytes x2: %s", bytes, hipGetErrorString(e));
        golhip_destroy(h);
        return code;
    }
    *out = h;
    return GOLHIP_OK;
}

// Alive count of this handle's rows at the current turn (h->mu held): the
// fused count of the last launch if it belongs to this turn, else a popcount.
int alive_count_locked(golhip_t h, uint64_t *count, int64_t *at_turn) {
    if (int rc = set_dev(h)) return rc;
    if (h->alive_turn != h->turns) {
        HIP_OR_FAIL(hipMemsetAsync(h->d_scalars, 0, sizeof(unsigned long long), h->stream));
        HIP_OR_FAIL(golk::launch_popcount(h->cur_rows(), h->local_words(), h->d_scalars, h->stream));
        h->alive_turn = h->turns;
    }
    HIP_OR_FAIL(hipMemcpyAsync(h->h_scalars, h->d_scalars, sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    *count = h->h_scalars[0];
    if (at_turn) *at_turn = h->alive_turn;
    return GOLHIP_OK;
}

// Grow-only device scratch (contents are not kept).
template <typename T>
int ensure_dev(golhip_t h, T **p, int64_t *cap, int64_t n, bool zero = false) {
    if (*cap >= n) return GOLHIP_OK;
    if (*p) HIP_OR_FAIL(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIP_OR_FAIL(hipMalloc((void **)p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    if (zero) HIP_OR_FAIL(hipMemsetAsync(*p, 0, (size_t)std::max<int64_t>(n, 1) * sizeof(T), h->stream));
    *cap = n;
    return GOLHIP_OK;
}

// The CellFlipped stream (distributor.go:93-173 with initializeAliveCells,
// :212-220): up to nturns single turns, each with its flip list appended in
// turn order to `out` (row-major within a turn; format: int32 (x, y) pairs or
// uint32 y * W + x).  stop: never lose an entry — the batch ends before the
// first turn whose list would not fit (the board is left at the last turn
// that did, *done says which); otherwise the board advances nturns and the
// lists are cut at cap (*total is what they needed).  counts[t] = entries
// of turn t, for t < *done.
int flip_stream_locked(golhip_t h, int64_t nturns, int format, void *out, uint64_t cap, uint64_t *counts,
                       int64_t *done_out, uint64_t *total_out, bool stop) {
    *done_out = 0;
    *total_out = 0;
    if (!h->loaded) return fail(GOLHIP_EINVAL, "no board loaded");
    if (h->nranks == 1 && !h->torus()) return fail(GOLHIP_EINVAL, "strip handle needs golhip_comm_init");
    if (int rc = set_dev(h)) return rc;
    h->flips_valid = false;
    if (nturns == 0) return GOLHIP_OK;
    const bool halo = h->ringed() && (h->nranks > 1 || h->force_halo);
    const int esz = format == GOLHIP_FLIPS_XY ? 8 : 4;
    const int64_t nw = h->local_words();
    const uint64_t most = (uint64_t)nturns * (uint64_t)h->W * (uint64_t)h->rows;
    const uint64_t dcap = std::min<uint64_t>({cap, most, (uint64_t)INT64_MAX / 16});
    if (int rc = ensure_dev(h, &h->d_run, &h->run_cap, nturns + 1)) return rc;
    std::vector<unsigned long long> run((size_t)nturns + 1, 0);
    unsigned ctl[2] = {0, 0};
    const int64_t t0 = h->turns;
    const int c0 = h->cur;

    if (h->W % 32 != 0 || nw >= (1ll << 32) - 4096) {
        // generic widths (the 16 x 16 fixture) and giant strips: the three-pass
        // compaction one turn at a time, checked on the host after each turn
        const int64_t nb = golk::compact_blocks(nw);
        if (int rc = ensure_blk(h, nb)) return rc;
        if (int rc = ensure_xy(h, (int64_t)std::min<uint64_t>(dcap, (uint64_t)nw * 32))) return rc;
        if (int rc = set_layout(h, want_il(h))) return rc;
        std::vector<int32_t> xy;
        int64_t t = 0;
        for (; t < nturns; ++t) {
            if (halo)
                if (int rc = exchange_rccl(h, 1, h->stream)) return rc;
            if (int rc = launch_depth(h, 1, t == nturns - 1, halo)) return rc;
            HIP_OR_FAIL(golk::launch_compact_count(h->cur_rows(), h->prev_rows(), nw, h->d_blk, h->stream));
            HIP_OR_FAIL(golk::launch_compact_scan(h->d_blk, nb, h->d_scalars + 1, h->stream));
            HIP_OR_FAIL(hipMemcpyAsync(h->h_scalars + 1, h->d_scalars + 1, 8, hipMemcpyDeviceToHost, h->stream));
            if (int rc = sync_stream(h)) return rc;
            const uint64_t k = h->h_scalars[1];
            if (stop && run[t] + k > dcap) {  // roll back this turn
                h->cur ^= 1;
                h->turns -= 1;
                h->alive_turn = -1;
                run[t + 1] = run[t] + k;
                break;
            }
            run[t + 1] = run[t] + k;
            const uint64_t keep = run[t] >= dcap ? 0 : std::min<uint64_t>(k, dcap - run[t]);
            if (keep > 0) {
                HIP_OR_FAIL(golk::launch_compact_scatter(h->cur_rows(), h->prev_rows(), nw, h->Ww, h->row0, h->d_blk,
                                                         h->d_xy, h->il, h->stream, (unsigned long long)h->xy_cap));
                xy.resize(2 * keep);
                HIP_OR_FAIL(hipMemcpyAsync(xy.data(), h->d_xy, keep * 8, hipMemcpyDeviceToHost, h->stream));
                if (int rc = sync_stream(h)) return rc;
                for (uint64_t e = 0; e < keep; ++e) {
                    if (format == GOLHIP_FLIPS_XY) {
                        static_cast<int32_t *>(out)[2 * (run[t] + e)] = xy[2 * e];
                        static_cast<int32_t *>(out)[2 * (run[t] + e) + 1] = xy[2 * e + 1];
                    } else {
                        static_cast<uint32_t *>(out)[run[t] + e] =
                            (uint32_t)((uint64_t)xy[2 * e + 1] * (uint64_t)h->W + (uint64_t)xy[2 * e]);
                    }
                }
            }
        }
        const int64_t done = t;
        for (int64_t i = 0; i < done; ++i) counts[i] = run[i + 1] - run[i];
        *done_out = done;
        *total_out = (stop && done < nturns) ? (done == 0 ? run[1] : run[done]) : run[done];
        return GOLHIP_OK;
    }

    // fused turn + list (K5) on the canonical layout; into a golhip_host_alloc
    // buffer the entries go without a host-side copy (option "flip_overlap"):
    //  2: K5r, the batch's turns in one resident launch whose copy blocks
    //     move each turn's list to the host while the next turns compute
    //     (round 6; where it cannot run: 1);
    //  1: each K5 launch's copy blocks move the previous turn's list;
    //  0: the turn's own blocks store their entries there directly
    if (int rc = set_layout(h, 0)) return rc;
    void *direct = mapped_device_ptr(out, (size_t)dcap * esz);
    const int64_t nb = golk::flip_turn_blocks(nw);
    const bool contig = h->Ww % 4 == 0;
    const int bpc = std::min(golk::flip_turn_blocks_per_cu(contig), 4);
    // every block resident at once (with a 10 % margin): block order = blockIdx.
    // Not in a multi-rank ring: its fallback (restore, re-run in ticket order)
    // would redo the batch's exchanges on this rank alone and hang the ring.
    const bool coresident = !h->ft_ticket && !(h->ringed() && h->nranks > 1) && bpc > 0 &&
                            nb * 10 <= (int64_t)h->cu_count * bpc * 9;
    // K5r: copy blocks in the slots the turn's blocks leave (up to 128), every
    // block resident; whole tori (a strip exchanges halos between turns);
    // buffers its 32-bit buffer offsets reach
    const int ncopy_r = (int)std::min<int64_t>(kFlipStreamCopyBlocks, (int64_t)h->cu_count * std::max(bpc, 1) - nb);
    const uint64_t board_bytes = (uint64_t)h->phys_rows * h->Ww * 4;
    // (A/B of handles a caller creates itself, e.g. the gol.Run mirror's:
    // GOLHIP_TUNING=1 GOLHIP_FLIP_OVERLAP=n overrides the option)
    if (const char *e = getenv("GOLHIP_FLIP_OVERLAP"); e && tuning_env() && e[0] >= '0' && e[0] <= '3' && !e[1])
        h->flip_overlap = e[0] - '0';
    if (const char *e = getenv("GOLHIP_FLIP_CP_GROUPS"); e && tuning_env() && e[0] >= '1' && e[0] <= '8' && !e[1])
        h->flip_cp_groups = e[0] - '0';
    // (boards under kFlipStreamMinBlocks blocks keep per-turn launches: their
    // lists are short, and K5r's per-turn waits cost more than a launch;
    // configs[0] through gol.Run measured within noise, profiles/r7u)
    const bool resident = direct && (h->flip_overlap == 3 || (h->flip_overlap == 2 && nb >= kFlipStreamMinBlocks)) &&
                          coresident && !halo && ncopy_r >= 8 &&
                          board_bytes < (1ull << 31) && (uint64_t)dcap * esz < (1ull << 31);
    const int ov = !direct ? 0 : resident ? 2 : std::min(h->flip_overlap, 1);
    const bool overlap = ov == 1;
    // launch the turns the buffer probably holds (the last batch's largest
    // list); turns past an overflow would only return at once
    int64_t nlaunch = nturns;
    if (stop && h->ft_est > 0) nlaunch = std::min<int64_t>(nturns, (int64_t)(dcap / h->ft_est) + 1);
    if (int rc = ensure_dev(h, &h->d_ftstatus, &h->ftstatus_cap, 3 * nb, true)) return rc;  // (K5r: three sets)
    if (int rc = ensure_dev(h, &h->d_ftticket, &h->ftticket_cap, nlaunch)) return rc;
    int64_t ctl_cap = h->d_ftctl ? 2 : 0;
    if (int rc = ensure_dev(h, &h->d_ftctl, &ctl_cap, 2)) return rc;
    if (!direct || ov) {
        int64_t bytes_cap = h->ev_cap_bytes;
        unsigned char *p = static_cast<unsigned char *>(h->d_ev);
        if (int rc = ensure_dev(h, &p, &bytes_cap, (int64_t)std::max<uint64_t>(dcap, 1) * esz)) return rc;
        h->d_ev = p;
        h->ev_cap_bytes = bytes_cap;
    }
    if (coresident) {  // keep the batch recoverable (see the error check below)
        const size_t bytes = (size_t)h->local_words() * 4;
        int64_t bcap = h->backup ? (int64_t)bytes : 0;
        if (int rc = ensure_dev(h, &h->backup, &bcap, h->local_words())) return rc;
        HIP_OR_FAIL(hipMemcpyAsync(h->backup, h->cur_rows(), bytes, hipMemcpyDeviceToDevice, h->stream));
    }
    // every run bound zeroed: a turn that never ran (after a stop) reads as an
    // empty list to the next launch's copy blocks
    HIP_OR_FAIL(hipMemsetAsync(h->d_run, 0, (size_t)(nlaunch + 1) * sizeof(unsigned long long), h->stream));
    // copy blocks: the slots the turn's blocks leave free (they come after
    // them in the grid, so the turn's blocks stay co-resident), 32..256
    const int cpb = overlap ? (int)std::max<int64_t>(32, std::min<int64_t>(256, (int64_t)h->cu_count * std::max(bpc, 1) - nb))
                            : 0;
    HIP_OR_FAIL(hipMemsetAsync(h->d_ftticket, 0, (size_t)nlaunch * sizeof(unsigned), h->stream));
    HIP_OR_FAIL(hipMemsetAsync(h->d_ftctl, 0, 2 * sizeof(unsigned), h->stream));
    golk::StepArgs sa = step_args(h, nullptr, halo);
    if (ov == 2 && nlaunch > 0) {
        // K5r: the whole batch in one launch (see FlipStreamArgs)
        // per turn kFtShards counters 128 B apart, then one turn count per compute block
        const int64_t ndone = nlaunch * golk::kFtShards * golk::kFtShardStride + nb;
        if (int rc = ensure_dev(h, &h->d_ftdone, &h->ftdone_cap, ndone)) return rc;
        HIP_OR_FAIL(hipMemsetAsync(h->d_ftdone, 0, (size_t)ndone * sizeof(unsigned), h->stream));
        HIP_OR_FAIL(hipMemsetAsync(h->d_scalars, 0, sizeof(unsigned long long), h->stream));
        golk::FlipStreamArgs fs{};
        golk::FlipTurnArgs &a = fs.turn;
        a.W = h->W;
        a.Ww = h->Ww;
        a.rows = h->rows;
        a.dst_base = kHalo;
        a.in = sa.in;
        a.row0 = h->row0;
        a.format = format == GOLHIP_FLIPS_XY ? golk::kFlipFormatXY : golk::kFlipFormatIdx;
        a.out = h->d_ev;
        a.ncompute = (int)nb;
        a.cap = dcap;
        a.status = h->d_ftstatus;
        a.ctl = h->d_ftctl;
        a.stop_on_overflow = stop ? 1 : 0;
        a.dbg = h->flip_debug;
        a.coresident = 1;
        a.board_bytes = (unsigned)board_bytes;
        a.out_bytes = (unsigned)((uint64_t)dcap * esz);
        fs.buf0 = h->buf[0];
        fs.buf1 = h->buf[1];
        fs.first = h->cur;
        fs.nturns = (int)nlaunch;
        // turn t's epoch is epoch0 + t: never 0 (the zeroed status words) in the batch
        if (((h->flip_epoch + 1) & 0x3FFFFFu) + (unsigned)nlaunch > 0x3FFFFFu) h->flip_epoch = 0;
        fs.epoch0 = (h->flip_epoch + 1) & 0x3FFFFFu;
        h->flip_epoch = (fs.epoch0 + (unsigned)nlaunch - 1) & 0x3FFFFFu;
        fs.run = h->d_run;
        fs.done = h->d_ftdone;
        fs.blk_done = h->d_ftdone + nlaunch * golk::kFtShards * golk::kFtShardStride;
        fs.alive = h->d_scalars;
        fs.cp_dst = direct;
        fs.ncopy = ncopy_r;
        fs.cp_groups = std::max(1, std::min(h->flip_cp_groups, ncopy_r / 8));
        fs.timeout_ticks = 200000000ll;  // 2 s: only a block that never became resident waits that long
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->flags & GOLHIP_FLAG_TIMING) {
            e0 = take_event(h);
            e1 = take_event(h);
            if (!e0 || !e1) return fail(GOLHIP_EHIP, "hipEventCreate failed");
            HIP_OR_FAIL(hipEventRecord(e0, h->stream));
        }
        HIP_OR_FAIL(golk::launch_flip_stream(fs, h->stream));
        if (e1) {
            HIP_OR_FAIL(hipEventRecord(e1, h->stream));
            h->ev_pending.push_back({e0, e1, 2});
        }
        h->flip_launches += nlaunch;
        h->flip_resident++;
        h->cur ^= (int)(nlaunch & 1);
        h->turns += nlaunch;
    }
    for (int64_t t = 0; ov != 2 && t < nlaunch; ++t) {
        if (halo)
            if (int rc = exchange_rccl(h, 1, h->stream)) return rc;
        const bool last = t == nlaunch - 1;
        if (last) HIP_OR_FAIL(hipMemsetAsync(h->d_scalars, 0, sizeof(unsigned long long), h->stream));
        golk::FlipTurnArgs a{};
        a.src = h->buf[h->cur];
        a.dst = h->buf[h->cur ^ 1];
        a.W = h->W;
        a.Ww = h->Ww;
        a.rows = h->rows;
        a.dst_base = kHalo;
        a.in = sa.in;
        a.row0 = h->row0;
        a.format = format == GOLHIP_FLIPS_XY ? golk::kFlipFormatXY : golk::kFlipFormatIdx;
        a.out = direct && !overlap ? direct : h->d_ev;
        a.ncompute = (int)nb;
        a.cp_run = overlap && t > 0 ? h->d_run + t - 1 : nullptr;
        a.cp_dst = direct;
        a.cp_blocks = cpb;
        a.cap = dcap;
        a.run = h->d_run + t;
        a.ticket = h->d_ftticket + t;
        a.status = h->d_ftstatus;
        h->flip_epoch = (h->flip_epoch + 1) & 0x3FFFFFu;
        if (h->flip_epoch == 0) h->flip_epoch = 1;  // 0 is the zeroed status array's epoch
        a.epoch = h->flip_epoch;
        a.ctl = h->d_ftctl;
        a.stop_on_overflow = stop ? 1 : 0;
        a.dbg = h->flip_debug;
        a.coresident = coresident ? 1 : 0;
        a.alive = last ? h->d_scalars : nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->flags & GOLHIP_FLAG_TIMING) {
            e0 = take_event(h);
            e1 = take_event(h);
            if (!e0 || !e1) return fail(GOLHIP_EHIP, "hipEventCreate failed");
            HIP_OR_FAIL(hipEventRecord(e0, h->stream));
        }
        HIP_OR_FAIL(golk::launch_flip_turn(a, h->stream));
        if (e1) {
            HIP_OR_FAIL(hipEventRecord(e1, h->stream));
            h->ev_pending.push_back({e0, e1, 2});
        }
        h->flip_launches++;
        h->cur ^= 1;
        h->turns += 1;
    }
    if (overlap && nlaunch > 0) {  // the last turn's list: a copy-only launch
        golk::FlipTurnArgs a{};
        a.Ww = h->Ww;
        a.format = format == GOLHIP_FLIPS_XY ? golk::kFlipFormatXY : golk::kFlipFormatIdx;
        a.out = h->d_ev;
        a.cap = dcap;
        a.ctl = h->d_ftctl;
        a.stop_on_overflow = stop ? 1 : 0;
        a.ncompute = 0;
        a.cp_run = h->d_run + nlaunch - 1;
        a.cp_dst = direct;
        a.cp_blocks = 256;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->flags & GOLHIP_FLAG_TIMING) {
            e0 = take_event(h);
            e1 = take_event(h);
            if (!e0 || !e1) return fail(GOLHIP_EHIP, "hipEventCreate failed");
            HIP_OR_FAIL(hipEventRecord(e0, h->stream));
        }
        HIP_OR_FAIL(golk::launch_flip_turn(a, h->stream));
        if (e1) {
            HIP_OR_FAIL(hipEventRecord(e1, h->stream));
            h->ev_pending.push_back({e0, e1, 2});
        }
    }
    HIP_OR_FAIL(hipMemcpyAsync(run.data(), h->d_run, (size_t)(nlaunch + 1) * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(ctl, h->d_ftctl, sizeof ctl, hipMemcpyDeviceToHost, h->stream));
    if (int rc = sync_stream(h)) return rc;
    for (auto &r : run) r &= ~golk::kFtRunReady;  // (K5r's ready bit)
    if (ctl[1]) {
        if (!coresident) return fail(GOLHIP_EHIP, "flip stream: look-back spin bound exceeded (board undefined)");
        // a block waited on a predecessor that never ran (a co-tenant kernel
        // held CUs): restore the batch's first board, re-run it in ticket order
        HIP_OR_FAIL(hipMemcpyAsync(h->buf[c0] + (int64_t)kHalo * h->Ww, h->backup, (size_t)h->local_words() * 4,
                                   hipMemcpyDeviceToDevice, h->stream));
        h->cur = c0;
        h->turns = t0;
        h->alive_turn = -1;
        h->ft_ticket = true;
        h->flip_fallbacks++;
        h->flip_debug &= ~4;
        return flip_stream_locked(h, nturns, format, out, cap, counts, done_out, total_out, stop);
    }
    int64_t done = nlaunch;
    if (stop)
        for (int64_t t = 0; t < nlaunch; ++t)
            if (run[t + 1] > dcap) {
                done = t;
                break;
            }
    if (done < nlaunch) {  // turn `done` overflowed and the later launches returned at once
        h->cur = (c0 + (int)(done & 1)) & 1;
        h->turns = t0 + done;
        h->alive_turn = -1;
    } else {
        h->alive_turn = h->turns;
    }
    uint64_t most_one = 0;
    for (int64_t t = 0; t < done; ++t) {
        counts[t] = run[t + 1] - run[t];
        most_one = std::max<uint64_t>(most_one, counts[t]);
    }
    if (done > 0) h->ft_est = most_one;
    const uint64_t total = done < nlaunch ? (done == 0 ? run[1] : run[done]) : run[nlaunch];
    const uint64_t got = done == 0 && stop ? 0 : std::min<uint64_t>(run[done], cap);
    if (got > 0 && !direct) {
        HIP_OR_FAIL(hipMemcpyAsync(out, h->d_ev, got * esz, hipMemcpyDeviceToHost, h->stream));
        if (int rc = sync_stream(h)) return rc;
    }
    h->flip_entries += (int64_t)got;
    *done_out = done;
    *total_out = total;
    return GOLHIP_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

const char *golhip_version(void) { return "golhip 0.1 (gfx950)"; }

const char *golhip_build_info(void) {
    static const std::string info = std::string(golk::build_info()) + kConsentInfo;
    return info.c_str();
}

const char *golhip_last_error(void) { return g_err.c_str(); }

int golhip_device_count(int32_t *n) {
    if (!n) return fail(GOLHIP_EINVAL, "n is null");
    int c = 0;
    HIP_OR_FAIL(hipGetDeviceCount(&c));
    *n = c;
    return GOLHIP_OK;
}

int golhip_host_alloc(uint64_t bytes, void **out) {
    if (!out || bytes == 0) return fail(GOLHIP_EINVAL, "bad host allocation");
    *out = nullptr;
    void *p = nullptr, *d = nullptr;
    hipError_t e = hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault);
    if (e != hipSuccess) return fail(GOLHIP_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(p);
        return fail(GOLHIP_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_bufs.push_back({(uintptr_t)p, (size_t)bytes, d});
    *out = p;
    return GOLHIP_OK;
}

int golhip_host_free(void *p) {
    if (!p) return GOLHIP_OK;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = std::find_if(g_host_bufs.begin(), g_host_bufs.end(),
                               [&](const HostBuf &b) { return b.base == (uintptr_t)p; });
        if (it == g_host_bufs.end()) return fail(GOLHIP_EINVAL, "not a golhip_host_alloc buffer");
        g_host_bufs.erase(it);
    }
    HIP_OR_FAIL(hipHostFree(p));
    return GOLHIP_OK;
}

int golhip_host_link_probe(int32_t device, uint64_t bytes, int32_t reps, double *kernel_write_gbps,
                           double *dma_d2h_gbps) {
    if (!kernel_write_gbps || !dma_d2h_gbps || bytes < 4096 || bytes % 16 || reps < 1 || reps > 1000)
        return fail(GOLHIP_EINVAL, "host link probe: bytes >= 4096, a multiple of 16; 1 <= reps <= 1000");
    *kernel_write_gbps = *dma_d2h_gbps = 0;
    HIP_OR_FAIL(hipSetDevice(device));
    int cus = 0;
    HIP_OR_FAIL(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    // the buffer K5 writes into: golhip_host_alloc's kind (hipHostMalloc, device-mapped)
    void *host = nullptr, *host_dev = nullptr, *dev = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipHostMalloc(&host, (size_t)bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&host_dev, host, 0);
    if (e == hipSuccess) e = hipMalloc(&dev, (size_t)bytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(dev, 0x5a, (size_t)bytes, st);
    // K5's own shape: 256-thread blocks, a few per CU, 16-byte stores
    const int blocks = 4 * cus;
    float kms = 0, dms = 0;
    if (e == hipSuccess) e = golk::launch_host_write_probe(host_dev, bytes, blocks, 0, st);  // warm (page mapping)
    if (e == hipSuccess) e = hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipEventRecord(e0, st);
    for (int r = 0; e == hipSuccess && r < reps; ++r) e = golk::launch_host_write_probe(host_dev, bytes, blocks, r + 1, st);
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&kms, e0, e1);
    if (e == hipSuccess) e = hipEventRecord(e0, st);
    for (int r = 0; e == hipSuccess && r < reps; ++r)
        e = hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&dms, e0, e1);
    // the last kernel pass's pattern must be in host memory (tag reps: word 0 == reps)
    if (e == hipSuccess && reps >= 1) {
        // (the DMA passes overwrote it with 0x5a bytes: check those instead)
        const uint32_t w = static_cast<const uint32_t *>(host)[bytes / 4 - 1];
        if (w != 0x5a5a5a5au) e = hipErrorUnknown;
    }
    if (e1) (void)hipEventDestroy(e1);
    if (e0) (void)hipEventDestroy(e0);
    if (st) (void)hipStreamDestroy(st);
    if (dev) (void)hipFree(dev);
    if (host) (void)hipHostFree(host);
    if (e != hipSuccess) return fail(GOLHIP_EHIP, "host link probe: %s", hipGetErrorString(e));
    *kernel_write_gbps = kms > 0 ? (double)bytes * reps / (kms * 1e-3) / 1e9 : 0;
    *dma_d2h_gbps = dms > 0 ? (double)bytes * reps / (dms * 1e-3) / 1e9 : 0;
    return GOLHIP_OK;
}

int golhip_create(int32_t width, int32_t height, int32_t device, uint32_t flags, golhip_t *out) {
    return create_common(width, height, 0, height, device, flags, false, out);
}

int golhip_create_strip(int32_t width, int32_t height, int32_t row0, int32_t rows, int32_t device, uint32_t flags,
                        golhip_t *out) {
    return create_common(width, height, row0, rows, device, flags, true, out);
}

int golhip_destroy(golhip_t h) {
    if (!h) return GOLHIP_OK;
    int rc = GOLHIP_OK;
    HIP_RC(hipSetDevice(h->device));
    if (h->stream) HIP_RC(hipStreamSynchronize(h->stream));
    for (auto &p : h->ev_pending) {
        HIP_RC(hipEventDestroy(p.e0));
        HIP_RC(hipEventDestroy(p.e1));
    }
    for (auto e : h->ev_pool) HIP_RC(hipEventDestroy(e));
    if (h->comm && ncclCommDestroy(h->comm) != ncclSuccess && rc == GOLHIP_OK)
        rc = fail(GOLHIP_ERCCL, "ncclCommDestroy failed");
    HIP_RC(hipFree(h->buf[0]));
    HIP_RC(hipFree(h->buf[1]));
    HIP_RC(hipFree(h->d_scalars));
    if (h->h_scalars) HIP_RC(hipHostFree(h->h_scalars));
    HIP_RC(hipFree(h->d_blk));
    HIP_RC(hipFree(h->d_xy));
    HIP_RC(hipFree(h->d_run));
    HIP_RC(hipFree(h->d_ftstatus));
    HIP_RC(hipFree(h->d_ftticket));
    HIP_RC(hipFree(h->d_ftctl));
    HIP_RC(hipFree(h->d_ftdone));
    HIP_RC(hipFree(h->d_ev));
    HIP_RC(hipFree(h->d_stage));
    HIP_RC(hipFree(h->d_sync));
    HIP_RC(hipFree(h->d_trace));
    HIP_RC(hipFree(h->backup));
    HIP_RC(hipFree(h->lds_edge));
    if (h->h_err) HIP_RC(hipHostFree(h->h_err));
    if (h->skew_err) HIP_RC(hipHostFree(h->skew_err));
    if (h->xport_host) HIP_RC(hipHostFree(h->xport_host));
    if (h->own_stream && h->stream) HIP_RC(hipStreamDestroy(h->stream));
    delete h;
    return rc;
}

int golhip_set_stream(golhip_t h, void *s) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (int rc_ = sync_stream(h)) return rc_;
    if (h->own_stream) HIP_OR_FAIL(hipStreamDestroy(h->stream));
    h->own_stream = false;
    h->stream = (hipStream_t)s;
    return GOLHIP_OK;
}

void *golhip_stream(golhip_t h) { return h ? (void *)h->stream : nullptr; }

int golhip_set_tb_depth(golhip_t h, int32_t t) {
    if (int rc = check(h)) return rc;
    if (t < 1 || t > GOLHIP_MAX_TB_DEPTH) return fail(GOLHIP_EINVAL, "tb depth %d not in 1..%d", t, GOLHIP_MAX_TB_DEPTH);
    std::lock_guard<std::mutex> g(h->mu);
    h->tb_depth = t;
    return GOLHIP_OK;
}

int golhip_set_rows_per_wave(golhip_t h, int32_t r) {
    if (int rc = check(h)) return rc;
    if (r < 0) return fail(GOLHIP_EINVAL, "rows per wave %d", r);
    std::lock_guard<std::mutex> g(h->mu);
    h->rows_per_wave = r;
    return GOLHIP_OK;
}

int golhip_set_option(golhip_t h, const char *key, int64_t value) {
    if (int rc = check(h)) return rc;
    if (!key) return fail(GOLHIP_EINVAL, "null option");
    for (const char *k : kTuningKeys)
        if (!strcmp(key, k) && !tuning_env())
            return fail(GOLHIP_EINVAL, "%s is an A/B tuning knob of the kernel plans: set GOLHIP_TUNING=1", key);
    std::lock_guard<std::mutex> g(h->mu);
    if (!strcmp(key, "resident_max_turns")) {  // test hook: several resident launches in one step
        if (value < 1 || value > golk::kResidentMaxTurns)
            return fail(GOLHIP_EINVAL, "resident_max_turns %lld", (long long)value);
        if (!test_hooks_env()) return fail(GOLHIP_EINVAL, "resident_max_turns is a test hook (GOLHIP_TEST_HOOKS=1)");
        h->resident_max = value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "wpl")) {
        if (value != 0 && value != 1 && value != 2 && value != 4)
            return fail(GOLHIP_EINVAL, "wpl %lld not in {0,1,2,4}", (long long)value);
        h->wpl_opt = (int)value;
        for (int &c : h->auto_rpw) c = 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persistent")) {
        if (value < -1 || value > 1) return fail(GOLHIP_EINVAL, "persistent %lld", (long long)value);
        h->persistent = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persist_depth")) {
        if (value < 0 || value > GOLHIP_MAX_TB_DEPTH) return fail(GOLHIP_EINVAL, "persist_depth %lld", (long long)value);
        h->persist_depth = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persist_waves")) {
        if (value != 0 && value != 4 && value != 8 && value != 16)
            return fail(GOLHIP_EINVAL, "persist_waves %lld not in {0,4,8,16}", (long long)value);
        h->persist_waves = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "dummy_rows")) {
        if (value < 0 || value > kHalo) return fail(GOLHIP_EINVAL, "dummy_rows %lld", (long long)value);
        h->dummy_rows = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "paired_bands")) {
        if (value < 0 || value > 1) return fail(GOLHIP_EINVAL, "paired_bands %lld", (long long)value);
        h->paired_bands = (int)value;
        for (int &c : h->auto_rpw) c = 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persist_half")) {
        if (value < 0 || value > 1) return fail(GOLHIP_EINVAL, "persist_half %lld", (long long)value);
        h->persist_half = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persist_wg_tx")) {
        if (value < 0 || value > 16) return fail(GOLHIP_EINVAL, "persist_wg_tx %lld", (long long)value);
        h->persist_wg_tx = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "trace")) {
        if (value && !h->d_trace) {
            if (hipMalloc(&h->d_trace, kTraceWords * sizeof(unsigned long long)) != hipSuccess)
                return fail(GOLHIP_ENOMEM, "trace buffer");
            if (hipMemsetAsync(h->d_trace, 0, kTraceWords * sizeof(unsigned long long), h->stream) != hipSuccess ||
                hipStreamSynchronize(h->stream) != hipSuccess)
                return fail(GOLHIP_EHIP, "trace buffer memset");
        }
        return GOLHIP_OK;
    }
    if (!strcmp(key, "persist_timeout_us")) {
        if (value < 1 || value > 60000000) return fail(GOLHIP_EINVAL, "persist_timeout_us %lld", (long long)value);
        h->persist_timeout_ticks = value * 100;  // s_memrealtime: 100 MHz
        return GOLHIP_OK;
    }
    if (!strcmp(key, "flip_debug")) {
        // 1 no look-back, 2 no entries (measurement only: wrong lists); 4 report a
        // co-residency failure once (tests the ticket-order fallback; lists exact)
        if (value < 0 || value > 7) return fail(GOLHIP_EINVAL, "flip_debug %lld", (long long)value);
        if ((value & 3) && !measurement_env())
            return fail(GOLHIP_EINVAL, "flip_debug %lld gives wrong lists: measurement runs only (GOLHIP_MEASUREMENT=1)",
                        (long long)value);
        if ((value & 4) && !test_hooks_env())
            return fail(GOLHIP_EINVAL, "flip_debug 4 is a test hook (GOLHIP_TEST_HOOKS=1)");
        h->flip_debug = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_pairs")) {
        if (value < 0 || value > 7) return fail(GOLHIP_EINVAL, "skew_pairs %lld", (long long)value);
        h->skew_pairs = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "flip_overlap")) {
        if (value < 0 || value > 3) return fail(GOLHIP_EINVAL, "flip_overlap %lld", (long long)value);
        h->flip_overlap = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "force_halo")) {
        h->force_halo = value != 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "cu_count")) {  // measurement: plan launches for fewer CUs (0: all of the device's)
        if (value < 0 || value > h->dev_cu) return fail(GOLHIP_EINVAL, "cu_count %lld not in 0..%d", (long long)value, h->dev_cu);
        h->cu_count = value ? (int)value : h->dev_cu;
        for (int &c : h->auto_rpw) c = 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "halo_skip")) {  // measurement only: the halo rows go stale (wrong results)
        if (value && !measurement_env())
            return fail(GOLHIP_EINVAL, "halo_skip gives wrong results: measurement runs only (GOLHIP_MEASUREMENT=1)");
        h->halo_skip = value != 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "fill_skip")) {
        h->fill_skip = value != 0;
        for (int &c : h->auto_rpw) c = 0;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew")) {
        if (value < 0 || value > 2) return fail(GOLHIP_EINVAL, "skew %lld", (long long)value);
        h->skew = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "timing")) {  // GOLHIP_FLAG_TIMING after creation (HIP events cost ~5 us a launch)
        if (value) h->flags |= GOLHIP_FLAG_TIMING;
        else h->flags &= ~GOLHIP_FLAG_TIMING;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_young")) {
        if (value != 0 && (value < 10 || value > 400))
            return fail(GOLHIP_EINVAL, "skew_young %lld not in 10..400", (long long)value);
        h->skew_young = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_hcap")) {
        if (value < -1 || value > 256) return fail(GOLHIP_EINVAL, "skew_hcap %lld", (long long)value);
        h->skew_hcap = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_prio")) {
        if (value < 0 || value > 1) return fail(GOLHIP_EINVAL, "skew_prio %lld", (long long)value);
        h->skew_prio = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_half")) {
        if (value < -1 || value > 1) return fail(GOLHIP_EINVAL, "skew_half %lld", (long long)value);
        h->skew_half = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "skew_tx")) {
        if (value < 0 || value > 2) return fail(GOLHIP_EINVAL, "skew_tx %lld", (long long)value);
        h->skew_tx = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_band")) {
        if (value < -1 || value > 1) return fail(GOLHIP_EINVAL, "lds_band %lld", (long long)value);
        h->lds_band = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_depth")) {
        if (value < 0 || value > 64) return fail(GOLHIP_EINVAL, "lds_depth %lld", (long long)value);
        h->lds_depth = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_waves")) {
        if (value != 0 && value != 8 && value != 16)
            return fail(GOLHIP_EINVAL, "lds_waves %lld not 0, 8 or 16", (long long)value);
        h->lds_waves = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_wg_cu")) {
        if (value < 1 || value > 2) return fail(GOLHIP_EINVAL, "lds_wg_cu %lld", (long long)value);
        h->lds_wg_cu = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_age")) {
        if (value != 0 && (value < 25 || value > 400)) return fail(GOLHIP_EINVAL, "lds_age %lld", (long long)value);
        h->lds_age = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_pre")) {
        if (value < 0 || value > 64) return fail(GOLHIP_EINVAL, "lds_pre %lld", (long long)value);
        h->lds_pre = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "resident_fault")) {
        if (value < 0 || value > 2) return fail(GOLHIP_EINVAL, "resident_fault %lld", (long long)value);
        if (value && !test_hooks_env())
            return fail(GOLHIP_EINVAL, "resident_fault is a test hook (GOLHIP_TEST_HOOKS=1)");
        h->resident_fault = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_stride")) {
        if (value < 0 || value > 1) return fail(GOLHIP_EINVAL, "lds_stride %lld", (long long)value);
        h->lds_stride = (int)value;
        return GOLHIP_OK;
    }
    if (!strcmp(key, "lds_xcd")) {
        if (value < 0 || value > 1) return fail(GOLHIP_EINVAL, "lds_xcd %lld", (long long)value);
        h->lds_xcd = (int)value;
        return GOLHIP_OK;
    }
    return fail(GOLHIP_EINVAL, "unknown option %s", key);
}

int golhip_comm_unique_id(uint8_t id[GOLHIP_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == GOLHIP_UNIQUE_ID_BYTES, "ncclUniqueId size");
    if (!id) return fail(GOLHIP_EINVAL, "id is null");
    ncclUniqueId u;
    NCCL_OR_FAIL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return GOLHIP_OK;
}

int golhip_comm_init(golhip_t h, const uint8_t id[GOLHIP_UNIQUE_ID_BYTES], int32_t nranks, int32_t rank) {
    if (int rc = check(h)) return rc;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(GOLHIP_EINVAL, "rank %d of %d", rank, nranks);
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (h->ringed()) return fail(GOLHIP_EINVAL, "comm already initialised");
    if (nranks > 1 && h->rows < 1) return fail(GOLHIP_EINVAL, "empty strip");
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    NCCL_OR_FAIL(ncclCommInitRank(&h->comm, nranks, u, rank));
    h->nranks = nranks;
    h->rank = rank;
    // agree on the schedule: the smallest strip of the ring
    int32_t *d_rows = nullptr;
    HIP_OR_FAIL(hipMalloc(&d_rows, sizeof(int32_t)));
    int32_t rows = h->rows;
    hipError_t e = hipMemcpyAsync(d_rows, &rows, sizeof rows, hipMemcpyHostToDevice, h->stream);
    ncclResult_t nr = e == hipSuccess ? ncclAllReduce(d_rows, d_rows, 1, ncclInt32, ncclMin, h->comm, h->stream) : ncclSuccess;
    if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpy(&rows, d_rows, sizeof rows, hipMemcpyDeviceToHost);
    (void)hipFree(d_rows);
    if (nr != ncclSuccess) return fail(GOLHIP_ERCCL, "ncclAllReduce(strip rows): %s", ncclGetErrorString(nr));
    if (e != hipSuccess) return fail(GOLHIP_EHIP, "strip rows: %s", hipGetErrorString(e));
    h->ring_rows = rows;
    return GOLHIP_OK;
}

int golhip_test_ring_init(golhip_t h, int32_t nranks, int32_t rank, int32_t ring_rows, golhip_test_transport_fn fn,
                          void *user) {
    if (int rc = check(h)) return rc;
    if (!test_hooks_env()) return fail(GOLHIP_EINVAL, "golhip_test_ring_init is a test hook: set GOLHIP_TEST_HOOKS=1");
    if (!fn || nranks < 1 || rank < 0 || rank >= nranks) return fail(GOLHIP_EINVAL, "rank %d of %d", rank, nranks);
    std::lock_guard<std::mutex> g(h->mu);
    if (h->ringed()) return fail(GOLHIP_EINVAL, "comm already initialised");
    if (!h->strip || h->rows < 1 || ring_rows < 1 || ring_rows > h->rows)
        return fail(GOLHIP_EINVAL, "a strip handle and 1 <= ring_rows <= its rows");
    h->xport = fn;
    h->xport_user = user;
    h->nranks = nranks;
    h->rank = rank;
    h->ring_rows = ring_rows;
    return GOLHIP_OK;
}

int golhip_comm_info(golhip_t h, int32_t *nranks, int32_t *rank, int32_t *ring_rows) {
    if (int rc = check(h)) return rc;
    if (!nranks || !rank || !ring_rows) return fail(GOLHIP_EINVAL, "null output");
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->comm) {  // no ring: this handle alone (or the test transport's ring)
        *nranks = h->xport ? h->nranks : 1;
        *rank = h->xport ? h->rank : 0;
        *ring_rows = h->xport ? h->ring_rows : h->rows;
        return GOLHIP_OK;
    }
    int n = 0, r = 0;
    NCCL_OR_FAIL(ncclCommCount(h->comm, &n));
    NCCL_OR_FAIL(ncclCommUserRank(h->comm, &r));
    *nranks = n;
    *rank = r;
    *ring_rows = h->ring_rows;
    return GOLHIP_OK;
}

int golhip_halo_schedule(int32_t strip_rows, int32_t tb_depth, int32_t resident, int64_t turns_left,
                         int32_t *depth, int32_t *launches) {
    if (!depth || !launches || strip_rows <= 0 || tb_depth < 1 || tb_depth > GOLHIP_MAX_TB_DEPTH || turns_left < 1)
        return fail(GOLHIP_EINVAL, "bad halo schedule request");
    const HaloRun hr = halo_next(std::min(tb_depth, strip_rows), strip_rows, resident != 0, turns_left);
    *depth = hr.d;
    *launches = hr.k;
    return GOLHIP_OK;
}

int golhip_halo_plan(int32_t width, int32_t strip_rows, int32_t nranks, int32_t rank, int32_t depth,
                     golhip_halo_plan_t *out) {
    if (!out || width <= 0 || strip_rows <= 0 || nranks < 1 || rank < 0 || rank >= nranks || depth < 1 ||
        depth > GOLHIP_HALO_ROWS || depth > strip_rows)
        return fail(GOLHIP_EINVAL, "bad halo plan request");
    plan(strip_rows, nranks, rank, depth, (width + 31) / 32, out);
    return GOLHIP_OK;
}

int golhip_load_bytes(golhip_t h, const uint8_t *cells) {
    if (int rc = check(h)) return rc;
    if (!cells) return fail(GOLHIP_EINVAL, "cells is null");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    const int64_t chunk = stage_rows(h);
    if (int rc = ensure_stage(h, chunk * h->W)) return rc;
    for (int64_t r = 0; r < h->rows; r += chunk) {
        const int64_t n = std::min<int64_t>(chunk, h->rows - r);
        HIP_OR_FAIL(hipMemcpyAsync(h->d_stage, cells + r * h->W, (size_t)(n * h->W), hipMemcpyHostToDevice, h->stream));
        HIP_OR_FAIL(golk::launch_pack(h->d_stage, h->cur_rows() + r * h->Ww, h->W, h->Ww, (int)n, h->stream));
    }
    if (int rc = loaded_canonical(h)) return rc;
    if (int rc_ = sync_stream(h)) return rc_;
    h->turns = 0;
    h->alive_turn = -1;
    h->flips_valid = false;
    return GOLHIP_OK;
}

int golhip_load_bits(golhip_t h, const uint32_t *words) {
    if (int rc = check(h)) return rc;
    if (!words) return fail(GOLHIP_EINVAL, "words is null");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    HIP_OR_FAIL(hipMemcpyAsync(h->cur_rows(), words, (size_t)h->local_words() * 4, hipMemcpyHostToDevice, h->stream));
    if (int rc = loaded_canonical(h)) return rc;
    if (int rc_ = sync_stream(h)) return rc_;
    h->turns = 0;
    h->alive_turn = -1;
    h->flips_valid = false;
    return GOLHIP_OK;
}

int golhip_fill_random(golhip_t h, uint64_t seed) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    HIP_OR_FAIL(golk::launch_fill_random(h->cur_rows(), h->W, h->Ww, h->rows, h->row0, seed, h->stream));
    if (int rc = loaded_canonical(h)) return rc;
    if (int rc_ = sync_stream(h)) return rc_;
    h->turns = 0;
    h->alive_turn = -1;
    h->flips_valid = false;
    return GOLHIP_OK;
}

}  // extern "C"

namespace {
// golhip_step with h->mu held.
int step_locked(golhip_t h, int64_t nturns, int32_t want_flips) {
    if (int rc = set_layout(h, want_il(h))) return rc;
    h->flips_valid = false;
    int64_t left = nturns;
    const int64_t tail = want_flips ? 1 : 0;
    // halo mode: row strips of a multi-rank ring, or (option force_halo) a
    // whole board run as a one-rank RCCL ring
    const bool halo = h->ringed() && (h->nranks > 1 || h->force_halo);
    if (!halo) {
        // resident launches while they apply (more than one only past
        // golk::kResidentMaxTurns turns), then per-launch kernels for the rest
        for (;;) {
            int rc = GOLHIP_OK;
            const int64_t n = try_persist(h, left - tail, tail == 0, &rc);
            if (rc) return rc;
            if (n <= 0) break;
            left -= n;
        }
    } else if (h->nranks == 1 && persist_on(h) && h->W % 32 == 0 && !h->guarded) {
        int rc = GOLHIP_OK;  // one-rank ring that may run resident launches: guard the step
        take_guard(h, &rc);
        if (rc) return rc;
    }
    while (left > tail) {
        if (!halo) {
            const int d = depth_plan(depth_cap(h, false), left - tail).d;
            if (int rc = launch_depth(h, d, left - d == 0, false)) return rc;
            left -= d;
            continue;
        }
        const HaloRun hr = halo_next(depth_cap(h, true), sched_rows(h), persist_on(h), left - tail);
        const int d = hr.d, k = hr.k;
        if (int rc = exchange_rccl(h, k * d, h->stream)) return rc;
        int prc = GOLHIP_OK;
        if (try_persist_halo(h, d, k, left - k * d == 0, &prc)) {
            left -= (int64_t)k * d;
            continue;
        }
        if (prc) return prc;
        for (int i = 0; i < k; ++i) {
            if (int rc = launch_ext(h, d, left - d == 0, (k - 1 - i) * d)) return rc;
            left -= d;
        }
    }
    if (want_flips && nturns > 0) {
        if (halo)
            if (int rc = exchange_rccl(h, 1, h->stream)) return rc;
        if (int rc = launch_depth(h, 1, true, halo)) return rc;
        if (int rc = start_flips(h)) return rc;
    }
    return GOLHIP_OK;
}
}  // namespace

extern "C" {

int golhip_step(golhip_t h, int64_t nturns, int32_t want_flips) {
    if (int rc = check(h)) return rc;
    if (nturns < 0) return fail(GOLHIP_EINVAL, "nturns %lld", (long long)nturns);
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->loaded) return fail(GOLHIP_EINVAL, "no board loaded");
    if (h->nranks == 1 && !h->torus()) return fail(GOLHIP_EINVAL, "strip handle needs golhip_comm_init or golhip_group_step");
    if (int rc = set_dev(h)) return rc;
    const int64_t turns0 = h->turns;
    const int cur0 = h->cur;
    // counters of this step, restored if a resident launch is abandoned below
    const int64_t persist_turns0 = h->persist_turns, persist_launches0 = h->persist_launches;
    const int64_t step_launches0 = h->step_launches, step_turns0 = h->step_turns;
    const int64_t skew_launches0 = h->skew_launches;
    const int64_t skew_half_launches0 = h->skew_half_launches, lds_launches0 = h->lds_launches;
    const int64_t pair_launches0 = h->pair_launches, pair_turns0 = h->pair_turns;
    const size_t ev0 = h->ev_pending.size();
    const int64_t halo_exchanges0 = h->halo_exchanges, halo_bytes0 = h->halo_bytes;
    int rc = step_locked(h, nturns, want_flips);
    const bool light = h->guard_light;
    h->guard_light = false;
    if (rc || !h->guarded) {
        h->guarded = false;
        return rc;
    }
    // A resident launch ran (torus, or a one-rank ring): check it before returning.  Its
    // workgroups wait on their neighbours, so a co-tenant kernel holding CUs
    // can starve one past the bounded spin; then every workgroup drains out
    // with the error word set and the board is restored from the guard copy
    // (the board before this step) and re-run on the per-launch kernels.
    h->guarded = false;
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    h->persist_pending = false;
    if (int rc_ = take_skew_err(h)) return rc_;
    if (!h->h_err || !*h->h_err) return GOLHIP_OK;  // (a one-rank ring's guard may see no resident launch)
    *h->h_err = 0;
    h->persistent = 0;  // this device is shared: no more resident launches on this handle
    h->persist_fallbacks++;
    h->persist_turns = persist_turns0;
    h->persist_launches = persist_launches0;
    h->step_launches = step_launches0;
    h->step_turns = step_turns0;
    h->skew_launches = skew_launches0;
    h->skew_half_launches = skew_half_launches0;
    h->lds_launches = lds_launches0;
    h->pair_launches = pair_launches0;
    h->pair_turns = pair_turns0;
    h->halo_exchanges = halo_exchanges0;
    h->halo_bytes = halo_bytes0;
    if (h->ev_pending.size() >= ev0) {  // the abandoned attempt's launch timings (unless drained meanwhile)
        for (size_t i = ev0; i < h->ev_pending.size(); ++i) {
            h->ev_pool.push_back(h->ev_pending[i].e0);
            h->ev_pool.push_back(h->ev_pending[i].e1);
        }
        h->ev_pending.resize(ev0);
    }
    if (!light)  // (a source-keeping launch left the step's board in buf[cur0])
        HIP_OR_FAIL(hipMemcpyAsync(h->buf[cur0] + (int64_t)kHalo * h->Ww, h->backup, (size_t)h->local_words() * 4,
                                   hipMemcpyDeviceToDevice, h->stream));
    h->cur = cur0;
    h->turns = turns0;
    h->alive_turn = -1;
    h->flips_valid = false;
    return step_locked(h, nturns, want_flips);
}

}  // extern "C"

namespace {
// golhip_group_step[_ex]: n strips (ring order = array order) driven from one
// process, halos moved by peer copies; want_flips keeps every strip's flip
// list of the last turn (golhip_flips, global coordinates, strip order =
// row-major order of the board).
int group_step_impl(golhip_t *hs, int32_t n, int64_t nturns, int32_t want_flips) {
    if (!hs || n < 1 || nturns < 0) return fail(GOLHIP_EINVAL, "bad group");
    for (int i = 0; i < n; ++i) {
        if (int rc = check(hs[i])) return rc;
        if (!hs[i]->loaded) return fail(GOLHIP_EINVAL, "strip %d has no board", i);
        if (hs[i]->W != hs[0]->W || hs[i]->H != hs[0]->H || hs[i]->nranks != 1)
            return fail(GOLHIP_EINVAL, "strip %d does not belong to the group", i);
        const int expect_row0 = i == 0 ? 0 : hs[i - 1]->row0 + hs[i - 1]->rows;
        if (hs[i]->row0 != expect_row0) return fail(GOLHIP_EINVAL, "strip %d starts at %d, expected %d", i, hs[i]->row0, expect_row0);
    }
    if (hs[n - 1]->row0 + hs[n - 1]->rows != hs[0]->H) return fail(GOLHIP_EINVAL, "strips do not cover the board");
    std::vector<std::unique_lock<std::mutex>> locks;
    for (int i = 0; i < n; ++i) locks.emplace_back(hs[i]->mu);
    std::vector<hipEvent_t> ready(n, nullptr);
    int rc = GOLHIP_OK;
    for (int i = 0; i < n; ++i) {
        HIP_RC(hipSetDevice(hs[i]->device));
        HIP_RC(hipEventCreateWithFlags(&ready[i], hipEventDisableTiming));
        if (!rc && want_il(hs[i]) != want_il(hs[0])) rc = fail(GOLHIP_EINVAL, "strip %d uses another word layout", i);
        if (!rc) rc = set_layout(hs[i], want_il(hs[i]));
        hs[i]->flips_valid = false;
    }
    // halo rows of every strip from its ring neighbours' current boards: x rows each way
    auto exchange = [&](int x) {
        for (int i = 0; i < n && !rc; ++i) {
            HIP_RC(hipSetDevice(hs[i]->device));
            HIP_RC(hipEventRecord(ready[i], hs[i]->stream));
        }
        for (int i = 0; i < n && !rc; ++i) {
            golhip *me = hs[i], *prev = hs[(i - 1 + n) % n], *next = hs[(i + 1) % n];
            golhip_halo_plan_t p;
            plan(me->rows, n, i, x, me->Ww, &p);
            HIP_RC(hipSetDevice(me->device));
            HIP_RC(hipStreamWaitEvent(me->stream, ready[(i - 1 + n) % n], 0));
            HIP_RC(hipStreamWaitEvent(me->stream, ready[(i + 1) % n], 0));
            const size_t bytes = (size_t)p.bytes;
            // top halo <- prev's last x rows; bottom halo <- next's first x rows
            uint32_t *mb = me->buf[me->cur];
            const uint32_t *pb = prev->buf[prev->cur] + (int64_t)(kHalo + prev->rows - x) * prev->Ww;
            const uint32_t *nb = next->buf[next->cur] + (int64_t)kHalo * next->Ww;
            HIP_RC(hipMemcpyPeerAsync(mb + (int64_t)p.recv_top_row * me->Ww, me->device, pb, prev->device, bytes,
                                      me->stream));
            HIP_RC(hipMemcpyPeerAsync(mb + (int64_t)p.recv_bottom_row * me->Ww, me->device, nb, next->device,
                                      bytes, me->stream));
            me->halo_bytes += 2 * (int64_t)bytes;
        }
        // a strip's second launch rewrites the buffer its neighbours copied
        // from: every stream waits for its neighbours' copies first
        for (int i = 0; i < n && !rc; ++i) {
            HIP_RC(hipSetDevice(hs[i]->device));
            HIP_RC(hipEventRecord(ready[i], hs[i]->stream));
        }
        for (int i = 0; i < n && !rc; ++i) {
            HIP_RC(hipSetDevice(hs[i]->device));
            HIP_RC(hipStreamWaitEvent(hs[i]->stream, ready[(i - 1 + n) % n], 0));
            HIP_RC(hipStreamWaitEvent(hs[i]->stream, ready[(i + 1) % n], 0));
        }
    };
    const int64_t tail = (want_flips && nturns > 0) ? 1 : 0;
    int64_t left = nturns - tail;
    while (left > 0 && rc == GOLHIP_OK) {
        int cap = GOLHIP_MAX_TB_DEPTH;
        for (int i = 0; i < n; ++i) cap = std::min(cap, depth_cap(hs[i], n > 1));
        const DepthRun run = depth_plan(cap, left);
        const int d = run.d;
        int k = 1;
        if (n > 1) {
            k = kHalo / d;
            for (int i = 0; i < n; ++i) k = std::min(k, halo_launches(hs[i]->rows, d, run.n));
            exchange(k * d);
        }
        for (int j = 0; j < k && rc == GOLHIP_OK; ++j) {
            for (int i = 0; i < n && !rc; ++i) {
                HIP_RC(hipSetDevice(hs[i]->device));
                if (rc) break;
                rc = n > 1 ? launch_ext(hs[i], d, left - d == 0, (k - 1 - j) * d)
                           : launch_depth(hs[i], d, left - d == 0, false);
            }
            left -= d;
        }
    }
    if (tail && rc == GOLHIP_OK) {  // the last turn alone, then its flip list on every strip
        if (n > 1) exchange(1);
        for (int i = 0; i < n && !rc; ++i) {
            HIP_RC(hipSetDevice(hs[i]->device));
            if (!rc) rc = n > 1 ? launch_ext(hs[i], 1, true, 0) : launch_depth(hs[i], 1, true, false);
            if (!rc) rc = start_flips(hs[i]);
        }
    }
    for (int i = 0; i < n; ++i) {
        HIP_RC(hipSetDevice(hs[i]->device));
        if (ready[i]) {
            HIP_RC(hipStreamSynchronize(hs[i]->stream));
            HIP_RC(hipEventDestroy(ready[i]));
        }
        if (!rc) rc = take_skew_err(hs[i]);
    }
    return rc;
}
}  // namespace

extern "C" {

int golhip_group_step(golhip_t *hs, int32_t n, int64_t nturns) { return group_step_impl(hs, n, nturns, 0); }

int golhip_group_step_ex(golhip_t *hs, int32_t n, int64_t nturns, int32_t want_flips) {
    return group_step_impl(hs, n, nturns, want_flips);
}

int golhip_sync(golhip_t h) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (int rc_ = sync_stream(h)) return rc_;
    return GOLHIP_OK;
}

int golhip_turn(golhip_t h, int64_t *t) {
    if (int rc = check(h)) return rc;
    if (!t) return fail(GOLHIP_EINVAL, "null out");
    *t = h->turns.load();
    return GOLHIP_OK;
}

int golhip_alive_count(golhip_t h, uint64_t *count, int64_t *at_turn) {
    if (int rc = check(h)) return rc;
    if (!count) return fail(GOLHIP_EINVAL, "null out");
    std::lock_guard<std::mutex> g(h->mu);
    return alive_count_locked(h, count, at_turn);
}

int golhip_alive_count_global(golhip_t h, uint64_t *count, int64_t *at_turn) {
    if (int rc = check(h)) return rc;
    if (!count) return fail(GOLHIP_EINVAL, "null out");
    // one critical section: local count, copy and allreduce all belong to the
    // same turn (a concurrent golhip_step cannot advance the board between them)
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = alive_count_locked(h, count, at_turn)) return rc;
    if (!h->ringed()) return GOLHIP_OK;
    if (!h->comm) {
        // test transport: the sum rides the same host callback (prev = next =
        // -1 marks an allreduce of one uint64, golhip_test_transport_fn)
        unsigned long long in = *count, out = 0;
        if (int r = h->xport(h->xport_user, -1, -1, &in, nullptr, &out, nullptr, (int64_t)sizeof in))
            return fail(GOLHIP_ERCCL, "test transport allreduce returned %d", r);
        *count = out;
        return GOLHIP_OK;
    }
    // the ring's RCCL communicator (also a one-rank ring: the same call as at 8 GPUs)
    HIP_OR_FAIL(hipMemcpyAsync(h->d_scalars + 3, h->d_scalars, sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                               h->stream));
    NCCL_OR_FAIL(ncclAllReduce(h->d_scalars + 3, h->d_scalars + 3, 1, ncclUint64, ncclSum, h->comm, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(h->h_scalars + 3, h->d_scalars + 3, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    *count = h->h_scalars[3];
    return GOLHIP_OK;
}

int golhip_flips(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (!h->flips_valid || h->flips_turn != h->turns) {
        if (n) *n = 0;
        return fail(GOLHIP_EINVAL, "no flip list: step with want_flips first");
    }
    return finish_compact(h, h->cur_rows(), h->prev_rows(), xy, cap, n);
}

int golhip_step_flips(golhip_t h, int64_t nturns, int32_t *xy, uint64_t cap, uint64_t *counts, uint64_t *n) {
    if (int rc = check(h)) return rc;
    if (n) *n = 0;
    if (nturns < 0) return fail(GOLHIP_EINVAL, "nturns %lld", (long long)nturns);
    if (nturns > 0 && !counts) return fail(GOLHIP_EINVAL, "counts is null");
    if (cap > 0 && !xy) return fail(GOLHIP_EINVAL, "xy is null");
    std::lock_guard<std::mutex> g(h->mu);
    // The flip kernel's look-back prefixes carry 40-bit offsets: run the batch
    // in chunks whose lists cannot reach 2^40 entries (every cell flipping
    // every turn), each appending after the last.
    const uint64_t cells = std::max<uint64_t>(1, (uint64_t)h->W * (uint64_t)h->rows);
    const int64_t chunk = std::max<int64_t>(1, (int64_t)((1ull << 40) / cells) - 1);
    uint64_t total = 0;
    for (int64_t t = 0; t < nturns || (t == 0 && nturns == 0);) {
        const int64_t m = std::min<int64_t>(chunk, nturns - t);
        const uint64_t got = std::min<uint64_t>(total, cap);
        int64_t done = 0;
        uint64_t part = 0;
        if (int rc = flip_stream_locked(h, m, GOLHIP_FLIPS_XY, xy ? xy + 2 * got : nullptr, cap - got, counts + t, &done,
                                        &part, false))
            return rc;
        total += part;
        t += m;
        if (m == 0) break;
    }
    if (n) *n = total;
    if (total > cap)
        return fail(GOLHIP_ERANGE, "buffer holds %llu cells, %llu needed", (unsigned long long)cap,
                    (unsigned long long)total);
    return GOLHIP_OK;
}

int golhip_flip_stream(golhip_t h, int64_t nturns, int32_t format, void *out, uint64_t cap, uint64_t *counts,
                       int64_t *turns_done, uint64_t *n) {
    if (int rc = check(h)) return rc;
    if (n) *n = 0;
    if (turns_done) *turns_done = 0;
    if (nturns < 0) return fail(GOLHIP_EINVAL, "nturns %lld", (long long)nturns);
    if (format != GOLHIP_FLIPS_XY && format != GOLHIP_FLIPS_INDEX) return fail(GOLHIP_EINVAL, "format %d", format);
    if (nturns > 0 && (!counts || !turns_done || !n)) return fail(GOLHIP_EINVAL, "counts / turns_done / n is null");
    if (cap > 0 && !out) return fail(GOLHIP_EINVAL, "out is null");
    if (format == GOLHIP_FLIPS_INDEX && (uint64_t)h->W * (uint64_t)h->H > (1ull << 32))
        return fail(GOLHIP_EINVAL, "cell indices of a %dx%d board do not fit in 32 bits", h->W, h->H);
    std::lock_guard<std::mutex> g(h->mu);
    if (h->ringed() && h->nranks > 1)
        return fail(GOLHIP_EINVAL, "golhip_flip_stream stops early on one rank alone: use golhip_step_flips in a ring");
    int64_t done = 0;
    uint64_t total = 0;
    if (int rc = flip_stream_locked(h, nturns, format, out, cap, counts, &done, &total, true)) return rc;
    *turns_done = done;
    *n = total;
    if (nturns > 0 && done == 0)
        return fail(GOLHIP_ERANGE, "buffer holds %llu entries, the next turn needs %llu", (unsigned long long)cap,
                    (unsigned long long)total);
    return GOLHIP_OK;
}

int golhip_alive_cells(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    const int64_t nw = h->local_words();
    const int64_t nb = golk::compact_blocks(nw);
    if (int rc = ensure_blk(h, nb)) return rc;
    HIP_OR_FAIL(golk::launch_compact_count(h->cur_rows(), nullptr, nw, h->d_blk, h->stream));
    HIP_OR_FAIL(golk::launch_compact_scan(h->d_blk, nb, h->d_scalars + 1, h->stream));
    h->flips_valid = false;  // d_blk reused
    return finish_compact(h, h->cur_rows(), nullptr, xy, cap, n);
}

int golhip_snapshot_bytes(golhip_t h, uint8_t *out) {
    if (int rc = check(h)) return rc;
    if (!out) return fail(GOLHIP_EINVAL, "out is null");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    const int64_t chunk = stage_rows(h);
    if (int rc = ensure_stage(h, chunk * h->W)) return rc;
    for (int64_t r = 0; r < h->rows; r += chunk) {
        const int64_t n = std::min<int64_t>(chunk, h->rows - r);
        HIP_OR_FAIL(golk::launch_unpack(h->cur_rows() + r * h->Ww, h->d_stage, h->W, h->Ww, (int)n, h->il, h->stream));
        HIP_OR_FAIL(hipMemcpyAsync(out + r * h->W, h->d_stage, (size_t)(n * h->W), hipMemcpyDeviceToHost, h->stream));
    }
    if (int rc_ = sync_stream(h)) return rc_;
    return GOLHIP_OK;
}

int golhip_snapshot_bits(golhip_t h, uint32_t *out) {
    if (int rc = check(h)) return rc;
    if (!out) return fail(GOLHIP_EINVAL, "out is null");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    const int il = h->il;
    HIP_OR_FAIL(golk::launch_convert_layout(h->cur_rows(), h->local_words(), il, 0, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(out, h->cur_rows(), (size_t)h->local_words() * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(golk::launch_convert_layout(h->cur_rows(), h->local_words(), 0, il, h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    return GOLHIP_OK;
}

int golhip_snapshot_rows(golhip_t h, int32_t row, int32_t nrows, uint32_t *out) {
    if (int rc = check(h)) return rc;
    if (!out || row < 0 || nrows < 0 || (int64_t)row + nrows > h->rows)
        return fail(GOLHIP_EINVAL, "rows [%d, %d) not in [0, %d)", row, row + nrows, h->rows);
    if (nrows == 0) return GOLHIP_OK;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    // a row holds whole pairs / quads in their layouts, so the range converts alone
    uint32_t *p = h->cur_rows() + (int64_t)row * h->Ww;
    const int64_t n = (int64_t)nrows * h->Ww;
    HIP_OR_FAIL(golk::launch_convert_layout(p, n, h->il, 0, h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(out, p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_OR_FAIL(golk::launch_convert_layout(p, n, 0, h->il, h->stream));
    return sync_stream(h);
}

int golhip_board_hash(golhip_t h, uint64_t *hash) {
    if (int rc = check(h)) return rc;
    if (!hash) return fail(GOLHIP_EINVAL, "null out");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    HIP_OR_FAIL(hipMemsetAsync(h->d_scalars + 2, 0, sizeof(unsigned long long), h->stream));
    HIP_OR_FAIL(golk::launch_hash(h->cur_rows(), h->local_words(), (int64_t)h->row0 * h->Ww, h->d_scalars + 2, h->il,
                                  h->stream));
    HIP_OR_FAIL(hipMemcpyAsync(h->h_scalars + 2, h->d_scalars + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               h->stream));
    if (int rc_ = sync_stream(h)) return rc_;
    *hash = h->h_scalars[2];
    return GOLHIP_OK;
}

int golhip_perf(golhip_t h, golhip_perf_t *out) {
    if (int rc = check(h)) return rc;
    if (!out) return fail(GOLHIP_EINVAL, "null out");
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (int rc = sync_stream(h)) return rc;
    if (int rc = drain_events(h)) return rc;
    memset(out, 0, sizeof *out);
    out->turns = h->turns;
    out->step_launches = h->step_launches;
    out->reserved1 = 0;  // retired kernel families (round 5): the fields stay for the ABI
    out->step_turns = h->step_turns;
    out->step_kernel_ms = h->step_ms;
    out->persist_launches = h->persist_launches;
    out->persist_turns = h->persist_turns;
    out->persist_kernel_ms = h->persist_ms;
    out->persist_fallbacks = h->persist_fallbacks;
    out->flip_launches = h->flip_launches;
    out->flip_kernel_ms = h->flip_ms;
    out->flip_entries = h->flip_entries;
    out->flip_fallbacks = h->flip_fallbacks;
    out->cell_updates = (int64_t)h->W * h->rows * (h->step_turns + h->persist_turns + h->flip_launches);
    out->alg_bytes = out->cell_updates / 4;
    out->halo_bytes = h->halo_bytes;
    const bool halo = h->ringed() && (h->nranks > 1 || h->force_halo);
    out->tb_depth = depth_cap(h, halo);
    out->rows_per_wave = rows_per_wave_for(h, next_depth(h, h->tb_depth, halo));
    out->kernel_variant = h->last_variant;
    out->skew_launches = h->skew_launches;
    out->halo_exchanges = h->halo_exchanges;
    out->halo_ms = h->halo_ms;
    out->reserved2 = 0;
    out->skew_half_launches = h->skew_half_launches;
    out->lds_launches = h->lds_launches;
    out->pair_launches = h->pair_launches;
    out->pair_turns = h->pair_turns;
    out->flip_resident_launches = h->flip_resident;
    out->words_per_lane = h->W % 32 == 0 ? wpl_for(h) : 0;
    out->persist_depth = h->W % 32 == 0 ? persist_depth_for(h, wpl_for(h)) : 0;
    return GOLHIP_OK;
}

int golhip_persist_trace_waves(golhip_t h, uint64_t *out, int64_t n) {
    if (int rc = check(h)) return rc;
    if (!out || n < 0 || n > kTraceWords - 8) return fail(GOLHIP_EINVAL, "bad out");
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->d_trace) return fail(GOLHIP_EINVAL, "set option \"trace\" first");
    if (int rc = set_dev(h)) return rc;
    if (int rc = sync_stream(h)) return rc;
    HIP_OR_FAIL(hipMemcpy(out, h->d_trace + 8, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return GOLHIP_OK;
}

int golhip_persist_trace(golhip_t h, uint64_t out[5]) {
    if (int rc = check(h)) return rc;
    if (!out) return fail(GOLHIP_EINVAL, "null out");
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->d_trace) return fail(GOLHIP_EINVAL, "set option \"trace\" first");
    if (int rc = set_dev(h)) return rc;
    if (int rc = sync_stream(h)) return rc;
    HIP_OR_FAIL(hipMemcpy(out, h->d_trace, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    HIP_OR_FAIL(hipMemsetAsync(h->d_trace, 0, 8 * sizeof(unsigned long long), h->stream));
    HIP_OR_FAIL(hipStreamSynchronize(h->stream));
    return GOLHIP_OK;
}

int golhip_perf_reset(golhip_t h) {
    if (int rc = check(h)) return rc;
    std::lock_guard<std::mutex> g(h->mu);
    if (int rc = set_dev(h)) return rc;
    if (int rc = drain_events(h)) return rc;
    h->step_ms = h->persist_ms = 0;
    h->step_launches = h->step_turns = h->halo_bytes = h->skew_launches = 0;
    h->persist_launches = h->persist_turns = 0;
    h->flip_launches = h->flip_entries = 0;
    h->flip_ms = 0;
    h->halo_exchanges = 0;
    h->halo_ms = 0;
    h->skew_half_launches = 0;
    h->lds_launches = 0;
    h->pair_launches = 0;
    h->pair_turns = 0;
    h->flip_resident = 0;
    return GOLHIP_OK;
}

}  // extern "C"
