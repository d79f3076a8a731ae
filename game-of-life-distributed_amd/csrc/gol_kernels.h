// gol_kernels.h — internal launchers for the gfx950 kernels of libgolhip.so.
// Not part of the C-ABI (include/golhip.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gol_limits.h"

namespace golk {

// Physical board buffers hold `rows + 2*kHalo` rows of Ww uint32 words; local
// row i lives at physical row kHalo + i.  Halo rows are filled by the ring
// exchange (strip mode) and unused in torus mode.
// Halo rows above and below a strip buffer (== GOLHIP_HALO_ROWS): deeper than
// one launch (GOLHIP_MAX_TB_DEPTH) so one exchange can feed several launches.
constexpr int kHalo = 128;
constexpr int kWave = 64;
constexpr int kTileValid = 62;   // lanes per wavefront tile that are stored (lanes 1..62)
constexpr int kHalfTileValid = 30;  // K1w half-wave tiles: lanes 1..30 of each 32-lane half

// How a step kernel finds input row i (logical, may be outside 0..rows-1).
//   torus mode : phys = base + mod(i, wrap)                 (whole board on one device)
//   halo  mode : phys = min(i + off, rmax)  (wrap == 0)     (row strip, halos filled)
struct RowMap {
    int base;
    int wrap;
    int off;
    int rmax;
};

struct StepArgs {
    const uint32_t *src;
    uint32_t *dst;
    int W;            // cells per row
    int Ww;           // words per row
    int rows_out;     // output rows (logical 0..rows_out-1)
    int dst_base;     // physical row of logical output row 0
    RowMap in;
    int rows_per_wave;
    int dummy_rows;   // >= 1 leading physical rows of dst usable as store dummies
    unsigned long long *alive;  // nullable: += popcount of the output rows [count_lo, count_hi)
    int count_lo, count_hi;
};

// Bit-sliced temporal-blocked step: `depth` in {1,2,4,8,16,32}; requires W % 32 == 0
// (wpl = 2: W % 64 == 0, depth <= 16, board in the interleaved pair layout).  fill_skip: skip the pipeline-fill
// stage-rows that only see padding.  wpl: words per lane (1 or 2).
hipError_t launch_step_tb(const StepArgs &a, int depth, hipStream_t s, bool fill_skip, int wpl, bool paired = false);
int max_depth_for(int wpl);
int persist_max_depth(int wpl);
int tb_tiles(int Ww, int wpl);
// One turn for any width (W % 32 != 0 boards such as 16x16).
hipError_t launch_step_generic(const StepArgs &a, hipStream_t s);
int tb_waves(const StepArgs &a, int wpl);
// Resident 256-thread blocks per CU of the depth-`depth` step kernel.
int tb_blocks_per_cu(int depth, int wpl);
int tb_wave_slots_per_cu(int depth, int wpl, bool paired);  // resident waves per CU
// Rows per wavefront minimising (rounds of waves) x (rows streamed per wave).
int auto_rows_per_wave(int Ww, int rows, int depth, int wave_slots, bool fill_skip, int wpl, bool paired = false);

// Skewed band stacks (K1w, gol_kernels.hip; torus and row strips, per
// launch).  Output rows [0, base.rows_out) of the StepArgs frame come from
// input rows [-D, rows_out + D) through base.in.  The input rows
// [-D, rows_out - D) split into nst stacks per tile column, one workgroup of
// 8 waves each = tx tiles x (8 / tx) bands; a band [a, e) of input rows owns
// generation g of the rows [a + g, e + g) (a parallelogram), so only the
// band below it feeds it (through LDS, from the top of that band's pipeline
// fill) and the stack's bottom band computes its own drain from the board.
struct SkewArgs {
    StepArgs base;
    int tiles_x;
    int tx;           // tiles per workgroup: 1 (stacks of 8 bands) or 2 (stacks of 4)
    int half;         // 1: half-wave tiles of 30 lanes (tiles_x counts them); each wave's upper lanes
                      //    run the same band of the stack rows_out / 2 further down (rows_out even)
    int nst;          // stacks per tile column
    int wgt[8];       // band heights by stack position (relative weights)
    int hcap;         // rows the stack's bottom band gives up (its drain is computed in full)
    int prio_young;   // 1: s_setprio 1 for waves 4..7 (the SIMD arbiter's age losers)
    unsigned *error;  // nullable, host-mapped: set if a band's imports never arrived (spin bound)
    unsigned long long *trace;  // nullable diagnostics: per wave (start, end) s_memrealtime at 8 + 2 (block * 64 + wave),
                                // (fill done, main loop done) at 8 + 2 (block * 64 + 8 + wave)
    int pairs;        // 1: the pair rule in the main loop (8 LUTs a word-turn; bands in multiples of 6 rows)
};
bool skew_supported(int depth, int wpl, bool half = false, bool pr = false);
int skew_blocks_per_cu(int depth, int wpl, bool half = false, bool pr = false);
hipError_t launch_skew(const SkewArgs &p, int depth, int wpl, hipStream_t s);

// Persistent multi-super-step step kernel (torus, or a strip's extended rows
// between two deep-halo exchanges); see gol_kernels.hip K1p.
struct PersistArgs {
    StepArgs base;            // rows_out, in-map, dst_base, W/Ww, alive (last super-step)
    uint32_t *buf0, *buf1;    // the two physical boards
    int first;                // buffer holding generation 0 (0 -> buf0)
    int J;                    // super-steps of `depth` turns
    int half_last;            // 1: the last super-step runs depth / 2 turns
    int S;                    // rows per wavefront
    int S_old, S_young;       // > 0: unequal bands, first / second half of the band rows (wg_sy even)
    int paired;               // 1: waves w, w + NW/2 share two bands, met from both ends (wg_sy even)
    int wg_tx, wg_sy;         // workgroup block of (tiles, strips)
    int cols, wg_y;           // workgroup grid
    int tiles_x;
    int nw;                   // waves per workgroup
    unsigned *progress;       // per workgroup, zeroed before launch
    unsigned *error;          // set on a spin timeout
    long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
    unsigned long long *trace; // nullable diagnostics (golhip_persist_trace)
    int fault;                // tests: workgroup 0 never reports progress (its neighbours time out)
};
int persist_waves_for(int depth, int wpl);
int persist_blocks_per_cu(int depth, int wpl, int nw);
// Workgroup shape / band height for `cus` resident workgroups of `units`
// (tile, strip) units each; false if none fits.  Caller sets p->nw.
// force_tx > 0: only workgroups of that many tiles across.
bool plan_persist(int Ww, int rows, int depth, int cus, int wpl, int units, PersistArgs *p, int force_tx = 0);
hipError_t launch_persist(const PersistArgs &p, int depth, int wpl, hipStream_t s);

// Resident LDS bands (K1r, gol_kernels.hip; small tori).  Workgroup b of nb
// keeps the full-width rows [b rows / nb, (b + 1) rows / nb) of the torus in
// LDS, with D halo rows on each side, and runs super-steps of D turns there;
// between super-steps it publishes its top and bottom D rows to `edge` and
// takes its neighbours' (write-through stores and loads, one flag per
// workgroup).  Every band needs >= D rows.  W % 128 == 0; wpl 1 (canonical
// words) or 2 (interleaved pairs).
struct LdsBandArgs {
    const uint32_t *src;   // generation 0: rows x Ww words
    uint32_t *dst;         // the last generation (the other buffer)
    uint32_t *edge;        // lds_band_edge_words(nb, D, Ww)
    unsigned *progress;    // nb words, zeroed: super-steps whose edges are published
    unsigned *error;       // zeroed; set on a spin timeout (every workgroup then drains)
    unsigned long long *alive;  // nullable: += popcount of the last generation
    long long timeout_ticks;    // s_memrealtime ticks (100 MHz) a wait may take
    int Ww, rows, nb, D, turns;
    int hmax;              // ceil(rows / nb)
    int xcd;               // 1: consecutive bands on one XCD (nb % 8 == 0)
    int nt;                // threads per workgroup: 512 or 1024
    int stride;            // LDS words per row: lds_band_stride (Ww; pairs Ww + 8, two planes)
    int rt_stride;         // 1: the runtime-stride kernel even where this stride is instantiated
    int fault;             // tests: band 0 never publishes, so its neighbours' waits time out
    int age;               // % row share of each younger wave rank against the next older one (100: equal
                           // runs; applies where whole waves fill a row's pairs, PC % 64 == 0)
    int pre;               // > 0: full super-steps run their first `pre` turns on the interior rows
                           //      while the halos travel (lds_pre)
    unsigned long long *trace;  // nullable: [0..3] += ticks in compute, publish, wait, halo load; [4] += workgroups
};
__host__ __device__ inline int64_t lds_band_edge_words(int nb, int D, int stride) { return 4ll * nb * D * stride; }
inline int64_t lds_band_lds_bytes(int hmax, int D, int stride) { return 2ll * (hmax + 2 * D + 3) * stride * 4; }
// Resident workgroups per CU at that LDS size (0: does not fit).
// The LDS row stride for Ww-word rows: Ww, pairs Ww + 8 (two planes with a ghost word each).
int lds_band_stride(int Ww, int wpl, int nt);
int lds_band_blocks_per_cu(int wpl, int nt, int stride, int64_t lds_bytes);
hipError_t launch_lds_band(const LdsBandArgs &p, int wpl, hipStream_t s);

hipError_t launch_pack(const uint8_t *bytes, uint32_t *words, int W, int Ww, int rows, hipStream_t s);
// il: the words are in the interleaved pair layout of the wpl = 2 step kernels
// (W % 64 == 0); pack / fill_random / load write canonical words, which the
// engine converts in place with launch_convert_layout.
hipError_t launch_unpack(const uint32_t *words, uint8_t *bytes, int W, int Ww, int rows, int il, hipStream_t s);
hipError_t launch_convert_layout(uint32_t *words, int64_t nwords, int from, int to, hipStream_t s);
hipError_t launch_fill_random(uint32_t *words, int W, int Ww, int rows, int64_t row0, uint64_t seed,
                              hipStream_t s);
hipError_t launch_popcount(const uint32_t *words, int64_t nwords, unsigned long long *out, hipStream_t s);
hipError_t launch_hash(const uint32_t *words, int64_t nwords, int64_t word0, unsigned long long *out, int il,
                       hipStream_t s);

// Row-major compaction of set bits of (a ^ b) (b nullable -> a alone) into
// (x, y) int32 pairs.  Three phases: per-block counts, one-block scan,
// ordered scatter.  compact_blocks() = per-block slots needed.  Batched
// lists (golhip_step_flips): `base` (device, nullable) offsets the scan so
// consecutive turns append, and the scatter drops pairs at index >= cap.
int64_t compact_blocks(int64_t nwords);
hipError_t launch_compact_count(const uint32_t *a, const uint32_t *b, int64_t nwords, unsigned long long *blk,
                                hipStream_t s);
hipError_t launch_compact_scan(unsigned long long *blk, int64_t nblk, unsigned long long *total, hipStream_t s,
                              const unsigned long long *base = nullptr);
hipError_t launch_compact_scatter(const uint32_t *a, const uint32_t *b, int64_t nwords, int Ww,
                                  int64_t row0, const unsigned long long *blk_off, int32_t *xy, int il,
                                  hipStream_t s, unsigned long long cap = ~0ull);

// K5: one turn fused with its CellFlipped list (golhip_flip_stream): each
// block steps 1024 consecutive words of the canonical board (W % 32 == 0),
// XORs old and new, finds its entries' offset with a single-pass decoupled
// look-back over the blocks, and writes its entries row-major through LDS.
// One launch per turn; the turn's lists append at run[0] and run[1] receives
// the running end.
constexpr int kFlipFormatXY = 0;   // int32 (x, y) pairs, 8 B per flip
constexpr int kFlipFormatIdx = 1;  // uint32 y * W + x, 4 B per flip
struct FlipTurnArgs {
    const uint32_t *src;
    uint32_t *dst;
    int W, Ww, rows;                // rows of this handle
    int dst_base;                   // physical row of local output row 0
    RowMap in;                      // input rows, as StepArgs::in
    long long row0;                 // global row of local row 0
    int format;                     // kFlipFormat*
    void *out;                      // entries (device)
    unsigned long long cap;         // entries that fit in out
    unsigned long long *run;        // run[0]: entries before this turn; run[1] <- after it
    unsigned *ticket;               // zeroed before the launch: virtual block ids
    unsigned long long *status;     // one look-back word per block
    unsigned epoch;                 // distinct for consecutive launches
    unsigned *ctl;                  // [0] stop: set by a turn that overflows cap (stop_on_overflow),
                                    //     every later launch returns at once; [1] error (spin bound)
    int stop_on_overflow;
    int dbg;                        // measurement only (option "flip_debug"): 1 no look-back, 2 no entries
    int coresident;                 // 1: the whole grid is resident at once (host-checked): block order is
                                    //    blockIdx and each block sums ALL its predecessors' aggregates;
                                    // 0: virtual ids from `ticket` and a decoupled look-back
    unsigned long long *alive;      // nullable: += popcount of the new board
    // Host copy of the PREVIOUS turn's list, overlapped with this turn (round
    // 6): cp_blocks extra blocks ahead of the turn's own (every block when the
    // launch is copy-only, ncompute 0) copy entries [cp_run[0], cp_run[1])
    // (cut at cap; none when stop_on_overflow and that turn overflowed) from
    // the device list `out` to the host list cp_dst (golhip_host_alloc memory).
    const unsigned long long *cp_run;  // nullable: no previous turn to copy
    void *cp_dst;
    int cp_blocks;
    int ncompute;                   // the turn's own blocks (flip_turn_blocks; 0: copy only)
    // K5r only (the sc1 hand-offs): the byte sizes of the board buffers and of `out`
    unsigned board_bytes, out_bytes;
    unsigned *done;                 // K5r: this turn's kFtShards done counters (kFtShardStride apart)
    unsigned *blk_done;             // K5r: per block, the turns it has finished
    unsigned turn;                  // K5r: this turn's index in the batch
};
int64_t flip_turn_blocks(int64_t nwords);
hipError_t launch_flip_turn(const FlipTurnArgs &a, hipStream_t s);
// K5r (flip_overlap 2, round 6): the turns of a flip-stream batch in ONE
// resident launch.  Compute blocks run K5's turn with a grid-wide wait
// between turns (the done counts of every block); copy blocks move each
// turn's list from the device list to the host list as soon as it is
// complete.  Every hand-off is write-through (sc1 stores drained by vmcnt,
// sc1 loads): no release or acquire fence, which on gfx950 would wait for
// the host writes in flight.
constexpr int kFtShards = 8;        // done counters a turn (arrivals spread over 8 words) ...
constexpr int kFtShardStride = 32;  // ... 128 bytes apart
// run[t + 1] as the last block stores it in K5r: the next turn's blocks wait
// for this bit (every reader, the host included, masks it off)
constexpr unsigned long long kFtRunReady = 1ull << 63;
struct FlipStreamArgs {
    FlipTurnArgs turn;              // per turn: src, dst, run, epoch, done, alive are set by the kernel
    uint32_t *buf0, *buf1;          // the handle's boards; turn t reads buf[(first + t) & 1]
    int first;
    int nturns;
    unsigned epoch0;                // turn t's look-back epoch: epoch0 + t (22 bits, never 0 in a batch)
    unsigned long long *run;        // run[t]: entries before turn t (run[0] = 0)
    unsigned *done;                 // done[kFtShards kFtShardStride t + kFtShardStride i] (zeroed)
    unsigned *blk_done;             // per compute block: turns finished (zeroed)
    unsigned long long *alive;      // nullable: the last turn's popcount
    void *cp_dst;                   // host list (device-mapped), the same offsets as turn.out
    int ncopy;                      // copy blocks (first in the grid)
    int cp_groups;                  // copy block c copies turns t = c mod cp_groups (mod cp_groups): one
                                    // group's turn-boundary gap (store acks, then loads) under another's stores
    long long timeout_ticks;        // one grid-wide wait (s_memrealtime, 100 MHz); past it: ctl[1]
};
hipError_t launch_flip_stream(const FlipStreamArgs &a, hipStream_t s);
int flip_turn_blocks_per_cu(bool contig);
// gol_probe.hip: coalesced 16-byte stores over `bytes` (a multiple of 16) of
// device-visible memory, e.g. page-locked host memory (the host-link probe)
hipError_t launch_host_write_probe(void *dst, uint64_t bytes, int blocks, uint32_t tag, hipStream_t s);

// "NAME=value ..." of the build's tuning macros (golhip_build_info).
const char *build_info();

}  // namespace golk
