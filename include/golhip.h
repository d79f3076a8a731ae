/*
 * golhip.h — C-ABI of libgolhip.so, the MI355X engine behind gol.Run.
 *
 * The reference's hot path is the per-turn loop of
 *   gol/distributor.go:93-173  distributor(): serial calculateNextState (:350-379)
 *                              or the worker pool worker/workerWorld (:304-347),
 *                              both over checkNeighbour (:382-417);
 * with its side channels
 *   gol/distributor.go:212-220 initializeAliveCells  -> CellFlipped events
 *   gol/distributor.go:420-432 calculateAliveCells   -> FinalTurnComplete.Alive,
 *                                                       AliveCellsCount (:283-302)
 *   gol/distributor.go:66-80   world fill from the io goroutine (ioInput)
 *   gol/distributor.go:180-191 final PGM stream (ioOutput), also s/q (:229-261).
 * The reference has no FFI of its own (pure Go); these entry points are what a
 * cgo shim in gol/distributor.go binds in place of those functions
 * (INTEGRATION.md shows the binding).  Plain pointers and sizes only.
 *
 * Board model: a width x height torus, rows are y (0..height-1), columns x.
 * Byte boards are row-major height x width, alive <=> byte == 255 (the
 * reference's test `world[x][y] == 255`, distributor.go:363, :411); byte
 * outputs are 0 / 255.  Bit boards are row-major, ceil(width/32) uint32 words
 * per row, cell (y, x) = bit x%32 of word x/32 (padding bits zero).
 *
 * Conventions: every function returns 0 (GOLHIP_OK) or a negative GOLHIP_E*
 * code and sets a thread-local message for golhip_last_error().  Caller-owned
 * buffers are never retained past the call (cgo pointer rules).  One handle is
 * driven by one engine thread; golhip_turn and golhip_alive_count may be
 * called concurrently from another thread (the reference's ticker, :283-302)
 * and return a (turn, count) pair that belongs together.
 */
#ifndef GOLHIP_H
#define GOLHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOLHIP_OK 0
#define GOLHIP_EINVAL (-1)  /* bad argument (size, pointer, state)            */
#define GOLHIP_EHIP (-2)    /* HIP runtime error                              */
#define GOLHIP_ENOMEM (-3)  /* device or host allocation failed               */
#define GOLHIP_ERANGE (-4)  /* caller buffer too small (required size is set) */
#define GOLHIP_ERCCL (-5)   /* RCCL error                                     */

/* golhip_create flags */
#define GOLHIP_FLAG_TIMING 0x1u /* time every step kernel with HIP events     */

#define GOLHIP_UNIQUE_ID_BYTES 128 /* == sizeof(ncclUniqueId)                 */
#define GOLHIP_MAX_TB_DEPTH 32     /* max turns fused in one step launch      */
#define GOLHIP_HALO_ROWS 128       /* halo rows above/below a strip buffer    */

typedef struct golhip golhip;
typedef golhip *golhip_t;

typedef struct golhip_perf {
    int64_t turns;            /* turns completed since the last load/fill     */
    int64_t step_launches;    /* per-launch step kernels (gol_tb_kernel) since golhip_perf_reset */
    int64_t step_turns;       /* turns run by those launches                  */
    double step_kernel_ms;    /* their summed device time (GOLHIP_FLAG_TIMING)*/
    int64_t persist_launches; /* persistent step kernels (gol_persist_kernel) */
    int64_t persist_turns;    /* turns run by those                           */
    double persist_kernel_ms; /* their summed device time (GOLHIP_FLAG_TIMING)*/
    int64_t cell_updates;     /* width * local rows * all stepped turns       */
    int64_t alg_bytes;        /* 0.25 B per cell-update (1 bit in + 1 bit out)*/
    int64_t halo_bytes;       /* bytes sent to neighbour ranks                */
    int32_t tb_depth;         /* most turns one step launch fuses (the setting,
                                 capped by the kernel's words per lane)       */
    int32_t rows_per_wave;    /* rows streamed per wavefront (full-depth launch)*/
    int32_t kernel_variant;   /* 0 = generic (width % 32 != 0), 1 = bit-sliced*/
    int32_t words_per_lane;   /* 1, 2 (interleaved pairs) or 4 (quads); 0 generic */
    int64_t persist_fallbacks; /* resident launches that timed out (not all workgroups
                                  co-resident) and were re-run on per-launch kernels */
    int64_t flip_launches;    /* fused turn + flip-list kernels (one turn each)  */
    int64_t flip_entries;     /* flip-list entries copied to the caller          */
    double flip_kernel_ms;    /* their summed device time (GOLHIP_FLAG_TIMING)   */
    int64_t flip_fallbacks;   /* flip batches re-run in ticket order (a block waited on a
                                 predecessor that was not resident)                */
    int32_t persist_depth;    /* turns per super-step of the resident kernel (its
                                 depths stop at 16 for two words per lane)       */
    int32_t reserved0;
    int64_t reserved1;        /* 0 (was split_launches: split tiling retired in round 5) */
    int64_t skew_launches;    /* of step_launches, those that ran skewed band
                                 stacks (gol_skew_kernel, kernel_variant 3)     */
    int64_t halo_exchanges;   /* halo exchanges posted (RCCL ring)               */
    double halo_ms;           /* their summed time on the stream they ran on
                                 (GOLHIP_FLAG_TIMING)                           */
    int64_t reserved2;        /* 0 (was overlap_launches: option "overlap" retired in round 5) */
    int64_t skew_half_launches; /* of skew_launches, those on half-wave tiles    */
    int64_t lds_launches;     /* of persist_launches, those that ran resident LDS
                                 bands (gol_lds_band_kernel, kernel_variant 4)  */
    int64_t pair_launches;    /* of skew_launches, those on the pair rule (option
                                 "skew_pairs": 8 LUTs a word-turn; round 6)     */
    int64_t pair_turns;       /* turns run by those                              */
    int64_t flip_resident_launches; /* flip-stream batches run as one resident launch
                                 (K5r, flip_overlap 2; round 6); their turns count in
                                 flip_launches, their time in flip_kernel_ms     */
} golhip_perf_t;

/* ---- library ---------------------------------------------------------- */
const char *golhip_version(void);
/* The build's kernel tuning macros, "NAME=value ..." (A/B builds override
 * them; the shipped library is built with the defaults).  Measurement. */
const char *golhip_build_info(void);
const char *golhip_last_error(void);
int golhip_device_count(int32_t *n);

/* Page-locked host memory that the device writes directly (hipHostMalloc,
 * mapped).  A golhip_flip_stream whose `out` lies inside such a buffer gets
 * its entries written by the kernels themselves over PCIe (each turn's list
 * by the next launch's copy blocks while that turn computes): no host-side
 * copy after the batch.  Go callers use it as C memory (unsafe.Slice). */
int golhip_host_alloc(uint64_t bytes, void **out);
int golhip_host_free(void *p);
/* Measurement (no reference counterpart): the host link's rates into a
 * buffer of golhip_host_alloc's kind -- a kernel streaming coalesced 16-byte
 * stores into it (what the event-stream kernel's entries ride) and the DMA
 * engine's device-to-host copy -- over `bytes` (>= 4096, a multiple of 16),
 * `reps` passes each after one warm pass, in GB/s (1e9 B/s). */
int golhip_host_link_probe(int32_t device, uint64_t bytes, int32_t reps, double *kernel_write_gbps,
                           double *dma_d2h_gbps);

/* ---- handles ---------------------------------------------------------- */
/* Whole width x height torus on one device.  Replaces the world allocation
 * of distributor.go:66-69. */
int golhip_create(int32_t width, int32_t height, int32_t device, uint32_t flags, golhip_t *out);

/* Row strip [row0, row0 + rows) of a width x height torus (multi-GPU row-strip
 * decomposition, README halo-exchange extension).  Its halo rows come from
 * the neighbouring strips through golhip_comm_init (one process per GPU, RCCL)
 * or golhip_group_step (several strips driven by one process). */
int golhip_create_strip(int32_t width, int32_t height, int32_t row0, int32_t rows, int32_t device,
                        uint32_t flags, golhip_t *out);
int golhip_destroy(golhip_t h);

/* Run on a caller-provided hipStream_t (e.g. torch.cuda.current_stream()). */
int golhip_set_stream(golhip_t h, void *hip_stream);
void *golhip_stream(golhip_t h);

/* Tuning: turns fused per launch (1..GOLHIP_MAX_TB_DEPTH, default 20; capped
 * per kernel: 32 at one word per lane, 20 at two (16 for the resident
 * kernel), 8 at four) and rows streamed
 * per wavefront (0 = automatic, the default: sized from the CU count and the
 * kernel's occupancy).  Results never depend on them. */
int golhip_set_tb_depth(golhip_t h, int32_t turns);
int golhip_set_rows_per_wave(golhip_t h, int32_t rows);
/* Named engine options; results never depend on them.
 *
 * Product options (no consent needed):
 * "wpl" (default 0 = auto): words per lane, 1, 2 or 4 (2 and 4 run on the
 *   interleaved pair / quad layouts, converted at the I/O boundary; 4 needs
 *   width % 128 == 0);
 * "persistent" (-1 = auto: off where the skewed band stacks fill the CUs,
 *   else on for buffers of at most 64 MiB; 1 on, 0 off): resident kernels
 *   (K1p, K1r) for long runs on a whole torus, never in a multi-rank ring --
 *   0 keeps a shared GPU free of kernels that wait on co-resident workgroups;
 * "lds_band" (-1 = auto, 1, 0): resident LDS bands (K1r, W % 128 == 0);
 * "skew" (1; 2 always, 0 off): skewed band stacks (K1w) for per-launch steps;
 * "timing" (GOLHIP_FLAG_TIMING after creation: per-launch HIP events);
 * "persist_timeout_us" (1000000): how long a resident workgroup waits for a
 *   neighbour before the launch is abandoned (the board is restored and the
 *   step re-run on per-launch kernels, perf.persist_fallbacks);
 * "force_halo" (0): after golhip_comm_init with one rank, run a whole board
 *   through the multi-GPU path as a one-rank RCCL ring.
 *
 * A/B tuning knobs of the kernel plans, refused without GOLHIP_TUNING=1 (or
 * GOLHIP_MEASUREMENT=1); the defaults are the measured plans:
 * persist_depth, persist_waves, persist_half, persist_wg_tx, paired_bands,
 * dummy_rows, trace (golhip_persist_trace), cu_count, fill_skip, skew_young,
 * skew_hcap, skew_prio, skew_half, skew_tx, lds_depth, lds_waves, lds_wg_cu,
 * lds_age, lds_pre, lds_stride, lds_xcd, skew_pairs (bit 1: tori and strips on
 * full-width K1w tiles run 18 turns a launch with the pair rule, 8 LUTs a
 * word-turn; bit 4: half-wave tile plans too; bit 2: quads at 8 on the pair
 * rule; default 5),
 * flip_overlap (how a golhip_flip_stream into golhip_host_alloc memory
 * delivers the lists: 2 (the default), boards of at least 64 K words run the
 * batch's turns as one resident launch whose copy blocks move each turn's
 * list to the host while the next turns compute, the rest (and whatever that
 * launch cannot run) as 1; 3, the resident launch at any size; 1, each
 * launch's copy blocks move the previous turn's list; 0, the turn's blocks
 * store their entries there).  Environment overrides for handles a caller
 * creates itself (GOLHIP_TUNING=1): GOLHIP_FLIP_OVERLAP=0..3, and
 * GOLHIP_FLIP_CP_GROUPS=1..8, the resident launch's copy-block groups (each
 * group copies every n-th turn; default 4).
 *
 * Measurement only, refused without GOLHIP_MEASUREMENT=1 (WRONG results by
 * design): "halo_skip" (post no halo exchange), "flip_debug" 1-3.
 *
 * Test hooks, refused without GOLHIP_TEST_HOOKS=1 (exact results, forced
 * failure paths): "resident_fault" (1: the resident kernels' band /
 * workgroup 0 never reports in any launch, 2: only in a step's first
 * resident launch; the neighbours' bounded waits time out and the step is
 * restored and re-run), "resident_max_turns" (lowers the turns one resident
 * launch takes, so a step runs several), "flip_debug" 4.
 *
 * golhip_build_info() lists the three consent sets and the product options.
 * Retired (refused as unknown keys): "split", "lds_split", "skew_nst",
 * "age_split", "overlap". */
int golhip_set_option(golhip_t h, const char *key, int64_t value);

/* ---- multi-GPU -------------------------------------------------------- */
/* RCCL ring of strips: rank r's neighbours are r-1 (rows above) and r+1
 * (rows below), mod nranks (toroidal wrap).  id comes from rank 0's
 * golhip_comm_unique_id, broadcast by the caller. */
int golhip_comm_unique_id(uint8_t id[GOLHIP_UNIQUE_ID_BYTES]);
int golhip_comm_init(golhip_t h, const uint8_t id[GOLHIP_UNIQUE_ID_BYTES], int32_t nranks, int32_t rank);
/* The ring as the communicator itself reports it (ncclCommCount /
 * ncclCommUserRank) and the strip rows every rank plans from (the ring's
 * smallest strip, agreed at golhip_comm_init).  Without a comm: 1, 0, and
 * this handle's rows.  No reference counterpart (measurement). */
int golhip_comm_info(golhip_t h, int32_t *nranks, int32_t *rank, int32_t *ring_rows);

/* Test hook, refused without GOLHIP_TEST_HOOKS=1 (no reference counterpart):
 * make a strip handle rank `rank` of an `nranks` ring whose halo exchange
 * runs through `fn` instead of RCCL, so that two processes can drive a ring
 * on one device.  At each exchange the library stages the strip's two send
 * blocks (its first and last `bytes / 4 / row words` rows beyond the halo
 * plan's send rows) in pinned memory and calls fn(user, prev_rank, next_rank,
 * send_up, send_down, recv_top, recv_bottom, bytes): fn must fill recv_top
 * with prev_rank's send_down and recv_bottom with next_rank's send_up, and
 * return 0.  Everything else (golhip_halo_schedule's rounds, the deep-halo
 * launches, the kernels) is the RCCL ring's; ring_rows is the ring's smallest
 * strip (golhip_comm_init agrees it by allreduce; here the caller passes it).
 * golhip_alive_count_global's allreduce runs through the same fn: prev_rank =
 * next_rank = -1, send_up = this rank's uint64 count, recv_top = where the
 * ring's sum goes, bytes = 8 (send_down, recv_bottom null). */
typedef int (*golhip_test_transport_fn)(void *user, int32_t prev_rank, int32_t next_rank, const void *send_up,
                                        const void *send_down, void *recv_top, void *recv_bottom, int64_t bytes);
int golhip_test_ring_init(golhip_t h, int32_t nranks, int32_t rank, int32_t ring_rows, golhip_test_transport_fn fn,
                          void *user);

/* Steps n strips (ring order = array order) driven from one process; halos
 * move with peer/device copies.  Same semantics as golhip_step on each. */
int golhip_group_step(golhip_t *hs, int32_t n, int64_t nturns);
/* golhip_group_step with golhip_step's want_flips: every strip keeps the flip
 * list of the last turn for golhip_flips (global coordinates; concatenated in
 * strip order they are the board's row-major list).  Used by gol.Run with
 * GOL_NGPU / GOL_STRIPS (the row-strip decomposition behind the drop-in). */
int golhip_group_step_ex(golhip_t *hs, int32_t n, int64_t nturns, int32_t want_flips);

/* Halo plan used by both transports (exposed for tests): rows this strip
 * sends up/down and receives for an exchange of `depth` rows
 * (1 <= depth <= min(GOLHIP_HALO_ROWS, strip_rows)). */
typedef struct golhip_halo_plan {
    int32_t prev_rank, next_rank;   /* ring neighbours                       */
    int32_t send_up_row, recv_top_row;     /* physical buffer rows             */
    int32_t send_down_row, recv_bottom_row;
    int32_t rows;                   /* = depth                               */
    int64_t bytes;                  /* per message                            */
} golhip_halo_plan_t;
int golhip_halo_plan(int32_t width, int32_t strip_rows, int32_t nranks, int32_t rank, int32_t depth,
                     golhip_halo_plan_t *out);
/* Exchange schedule of a strip, exactly as golhip_step runs it: each
 * exchange moves launches * depth halo rows, then `launches` step launches of
 * `depth` turns follow; launch i (0-based) steps rows [-e, strip_rows + e),
 * e = (launches - 1 - i) * depth, so it rebuilds the next launch's halos from
 * the deeper exchanged ones (kernel-side rows, W % 32 == 0; other widths run
 * one turn per launch).  tb_depth: the most turns a launch may fuse (the
 * setting capped by the kernel's words per lane, golhip_perf tb_depth);
 * resident != 0: the strip runs the resident kernel between exchanges
 * (option "persistent", on by default for strips of <= 64 MiB), which takes
 * full-depth super-steps greedily instead of the balanced launch plan. */
int golhip_halo_schedule(int32_t strip_rows, int32_t tb_depth, int32_t resident, int64_t turns_left,
                         int32_t *depth, int32_t *launches);

/* ---- board I/O -------------------------------------------------------- */
/* Load this handle's rows (height x width bytes, or its strip's rows). */
int golhip_load_bytes(golhip_t h, const uint8_t *cells);
int golhip_load_bits(golhip_t h, const uint32_t *words);
/* Synthetic board: cell (y, x) alive <=> (splitmix64(seed ^ (y*width + x)) & 3) == 0,
 * global coordinates (strips of one board agree). */
int golhip_fill_random(golhip_t h, uint64_t seed);

/* ---- the turn loop ---------------------------------------------------- */
/* Enqueue nturns turns (asynchronous).  want_flips != 0 keeps the flip list
 * of the LAST turn for golhip_flips (initializeAliveCells, :212-220). */
int golhip_step(golhip_t h, int64_t nturns, int32_t want_flips);
int golhip_sync(golhip_t h);
int golhip_turn(golhip_t h, int64_t *turns_done);

/* ---- side channels ---------------------------------------------------- */
/* Alive cells of this handle's rows at turn *at_turn (len(calculateAliveCells)). */
int golhip_alive_count(golhip_t h, uint64_t *count, int64_t *at_turn);
/* Sum over the RCCL ring (equals golhip_alive_count without a comm). */
int golhip_alive_count_global(golhip_t h, uint64_t *count, int64_t *at_turn);
/* Cells that changed in the last stepped turn (want_flips), row-major,
 * (x = col, y = row) pairs in global coordinates.  ERANGE sets *n. */
int golhip_flips(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n);
/* Batched CellFlipped stream (distributor.go:93-173 with the per-turn
 * initializeAliveCells :212-220): advance nturns turns one at a time and
 * return every turn's flip list, concatenated in turn order (row-major within
 * a turn, same pairs as golhip_flips), with counts[t] = flips of turn t.
 * One host round trip for the whole batch, on the fused turn + list kernel
 * (K5).  The board always advances nturns; if the lists exceed cap pairs, xy
 * holds the first cap, *n the total and the call returns GOLHIP_ERANGE.
 * Reserves min(cap, nturns x cells) pairs on the device.  Works in a
 * multi-rank ring; golhip_flip_stream (below) never drops a flip. */
int golhip_step_flips(golhip_t h, int64_t nturns, int32_t *xy, uint64_t cap, uint64_t *counts, uint64_t *n);
/* The CellFlipped stream without loss: advance UP TO nturns turns, one at a
 * time, each fused with its flip list on the device (initializeAliveCells,
 * :212-220), and append the lists in turn order to `out` (row-major within a
 * turn): format GOLHIP_FLIPS_XY = int32 (x = col, y = row) pairs, 8 bytes a
 * flip; GOLHIP_FLIPS_INDEX = uint32 y * width + x, 4 bytes a flip (boards of
 * at most 2^32 cells).  cap counts entries.  The batch stops before the
 * first turn whose list would not fit, so no flip is ever dropped: the board
 * is left at the last turn that fitted, *turns_done says how many ran
 * (counts[t] for t < *turns_done), *n = entries written.  If not even the
 * first turn fits: GOLHIP_ERANGE, nothing advanced, *n = entries it needs.
 * One host round trip per call.  Not for multi-rank rings (a stop on one
 * rank would desynchronise them): use golhip_step_flips there. */
#define GOLHIP_FLIPS_XY 0
#define GOLHIP_FLIPS_INDEX 1
int golhip_flip_stream(golhip_t h, int64_t nturns, int32_t format, void *out, uint64_t cap, uint64_t *counts,
                       int64_t *turns_done, uint64_t *n);
/* Alive cells, row-major (x = col, y = row) pairs — calculateAliveCells. */
int golhip_alive_cells(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n);
/* Board as 0/255 bytes / bit words (this handle's rows). */
int golhip_snapshot_bytes(golhip_t h, uint8_t *out);
int golhip_snapshot_bits(golhip_t h, uint32_t *out);
/* Bit words of rows [row, row + nrows) of this handle (nrows x ceil(width/32)
 * uint32): a few rows of a board too large to copy whole (the 262144^2
 * full-size checks). */
int golhip_snapshot_rows(golhip_t h, int32_t row, int32_t nrows, uint32_t *out);
/* Order-independent board digest: sum over words of
 * splitmix64((global_word_index << 32) | word) mod 2^64 (strips add up). */
int golhip_board_hash(golhip_t h, uint64_t *hash);

/* ---- measurement ------------------------------------------------------ */
int golhip_perf(golhip_t h, golhip_perf_t *out);
/* Diagnostics of the persistent step kernels since the last call (option
 * "trace" must be set before stepping): out[0] = sum over waves of band
 * compute time, out[1] = longest band of one super-step, out[2] = sum over
 * workgroups of time spent waiting for neighbour workgroups, out[3] = sum
 * over workgroups of kernel time, out[4] = workgroup count; times in
 * s_memrealtime ticks (100 MHz).  No reference counterpart (measurement). */
int golhip_persist_trace(golhip_t h, uint64_t out[5]);
/* Per-wave (start, end) ticks of the middle super-step of the last persistent
 * launch: out[2 * (workgroup * 64 + wave) + {0, 1}], n words. */
int golhip_persist_trace_waves(golhip_t h, uint64_t *out, int64_t n);
int golhip_perf_reset(golhip_t h);

#ifdef __cplusplus
}
#endif
#endif /* GOLHIP_H */
