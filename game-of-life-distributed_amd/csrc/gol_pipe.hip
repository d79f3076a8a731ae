// gol_pipe.hip — K1t, the resident LDS turn pipeline of libgolhip.so (small
// tori whose rows are one wavefront wide); see gol_kernels.h PipeArgs.
#include "gol_kernels.h"
#include "gol_bits.h"

#include <type_traits>
#include <utility>

namespace golk {

// ---------------------------------------------------------------------------
// K1t: resident LDS turn pipeline (round 5; small tori whose rows are one
// wavefront wide, Ww == 64 * WPL: 2048 (WPL 1), 4096 (pairs), 8192 (quads)).
//
// K1r recomputes a D-row trapezoid at both ends of every band each
// super-step, hands the halos over with a grid-wide flag protocol every D
// turns and runs one workgroup barrier per turn.  K1t removes all three:
//  * skewed bands: generation t of band b is the rows [r_b + t, r_{b+1} + t)
//    (mod rows), so its row i needs generation t - 1's rows i, i + 1, i + 2;
//    rows h, h + 1 are the band below's first two rows of generation t - 1.
//    Every row is computed once and the only import is two rows per turn
//    from the band below, produced at the start of that band's stream and
//    needed at the end of ours (h rows of slack);
//  * one wave per turn: wave w computes the turns w + 1, w + 1 + S, ... (S =
//    kPipeWaves): it streams the rows of its band top to bottom, reading the
//    previous turn's rows from the previous wave's LDS ring and writing its
//    own into its ring; the last wave's ring feeds the first wave's next
//    turn, so the turns circulate through the workgroup with no barrier;
//  * a whole torus row per wave: horizontal neighbours come from the adjacent
//    lanes by DPP wave rotates (lane 63 <-> lane 0 is the column wrap), so
//    there are no halo lanes and no LDS neighbour reads.
// Ring hand-off: the producer writes the row (all lanes) and then the slot's
// tag = sequence + 1 (one lane); the consumer reads the tag and then the row
// and retries while the tag is old.  A wave's LDS operations execute in
// order, so a new tag implies the row before it.  The consumer publishes
// how many rows it has read (CONS); the producer reuses a slot only after.
// Edges (rows 0 and 1 of each turn but the last) go to global memory with
// write-through stores, then a flag = the turn (after the wave's vmcnt(0));
// the band above polls the flag with sc1 loads early in its turn and loads
// the two rows with sc1 loads (MI355X_MICROARCH.md hand-off table, row 1),
// then reports the turn read (econs), which bounds how far a band may run
// ahead of the band above (kPipeQ edge slots).  Every wait is bounded: a
// timeout sets the error word, every wave drains, and the host restores the
// board and re-runs the step on per-launch kernels (as for K1r / K1p).
// Per row and word: 9 LUTs + the shifts (WPL 4: 1/2 DPP + 1/2 alignbit per
// word); per row a 16-B (quads) LDS read and write.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) {  // lane i <- lane i - 1, lane 0 <- lane 63
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_rol1(uint32_t v) {  // lane i <- lane i + 1, lane 63 <- lane 0
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, false);
}
// Row sums of a whole torus row held by one wave (the row wraps across lanes).
template <int WPL>
__device__ __forceinline__ void pipe_sums(const uint32_t (&x)[WPL], LdsRow<WPL> &s) {
    uint32_t west[WPL], east[WPL];
    if constexpr (WPL == 1) {
        west[0] = __builtin_amdgcn_alignbit(x[0], wave_ror1(x[0]), 31);
        east[0] = __builtin_amdgcn_alignbit(wave_rol1(x[0]), x[0], 1);
    } else if constexpr (WPL == 2) {
        west[0] = __builtin_amdgcn_alignbit(x[1], wave_ror1(x[1]), 31);  // cell 2k - 1
        east[0] = x[1];
        west[1] = x[0];
        east[1] = __builtin_amdgcn_alignbit(wave_rol1(x[0]), x[0], 1);   // cell 2k + 2
    } else {
        west[0] = __builtin_amdgcn_alignbit(x[3], wave_ror1(x[3]), 31);  // cell 4k - 1
        west[1] = x[0];
        west[2] = x[1];
        west[3] = x[2];
        east[0] = x[1];
        east[1] = x[2];
        east[2] = x[3];
        east[3] = __builtin_amdgcn_alignbit(wave_rol1(x[0]), x[0], 1);   // cell 4k + 4
    }
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        s.c[k] = x[k];
        s.s0[k] = bop<kXor3>(west[k], x[k], east[k]);
        s.s1[k] = bop<kMaj>(west[k], x[k], east[k]);
    }
}
template <int WPL>
struct PipeRaw {
    uint32_t w[WPL];
    uint32_t tag;
};
template <int WPL>
__device__ __forceinline__ void lanes_load(const uint32_t *p, uint32_t (&v)[WPL]) {
    if constexpr (WPL == 1) {
        v[0] = *p;
    } else if constexpr (WPL == 2) {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        v[0] = q.x;
        v[1] = q.y;
    } else {
        const uint4 q = *reinterpret_cast<const uint4 *>(p);
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    }
}
template <int WPL>
__device__ __forceinline__ void lanes_store(uint32_t *p, const uint32_t (&v)[WPL]) {
    if constexpr (WPL == 1)
        *p = v[0];
    else if constexpr (WPL == 2)
        *reinterpret_cast<uint2 *>(p) = make_uint2(v[0], v[1]);
    else
        *reinterpret_cast<uint4 *>(p) = make_uint4(v[0], v[1], v[2], v[3]);
}
// sc1 (L1-bypassing / write-through) buffer accesses of WPL words at byte offset `off`
template <int WPL>
__device__ __forceinline__ void buf_load_sc1(__amdgpu_buffer_rsrc_t rs, int off, uint32_t (&v)[WPL]) {
    if constexpr (WPL == 1) {
        v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, kCpolSc1);
    } else if constexpr (WPL == 2) {
        typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
        const v2u32 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, kCpolSc1);
        v[0] = q.x;
        v[1] = q.y;
    } else {
        const v4u32 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kCpolSc1);
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    }
}
template <int WPL>
__device__ __forceinline__ void buf_store_sc1(__amdgpu_buffer_rsrc_t rs, int off, const uint32_t (&v)[WPL]) {
    if constexpr (WPL == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(v[0], rs, off, 0, kCpolSc1);
    } else if constexpr (WPL == 2) {
        typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((v2u32){v[0], v[1]}, rs, off, 0, kCpolSc1);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128((v4u32){v[0], v[1], v[2], v[3]}, rs, off, 0, kCpolSc1);
    }
}
#define GOL_CBAR() asm volatile("" ::: "memory")  // no compiler reordering of memory operations across

// Edge rows as 8-byte {word, tag} granules, each written by one sc1 store
// and read by one sc1 load (MI355X_MICROARCH.md, hand-off table: a granule is
// seen whole): no flag, no drain wait on the producer, one round trip for
// the consumer.  Lane L's WPL granules of edge row r sit at byte
// ((row index) * 64 + L) * WPL * 8.
// (kept as the loaded vectors: picking the words out into registers of
// their own made the compiler wait for the loads where they were issued)
template <int WPL>
struct Gran {
    static constexpr int N = WPL == 1 ? 1 : WPL / 2;  // 8-B (WPL 1) or 16-B loads
    typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
    typedef typename std::conditional<WPL == 1, v2u32, v4u32>::type V;
    V v[N];
    __device__ __forceinline__ uint32_t word(int k) const {
        if constexpr (WPL == 1) return v[0].x;
        else return (k & 1) ? v[k >> 1].z : v[k >> 1].x;
    }
    __device__ __forceinline__ uint32_t tag(int k) const {
        if constexpr (WPL == 1) return v[0].y;
        else return (k & 1) ? v[k >> 1].w : v[k >> 1].y;
    }
};
template <int WPL>
__device__ __forceinline__ void gran_store(__amdgpu_buffer_rsrc_t rs, int off, const uint32_t (&v)[WPL], uint32_t tag) {
    typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
    if constexpr (WPL == 1) {
        __builtin_amdgcn_raw_buffer_store_b64((v2u32){v[0], tag}, rs, off, 0, kCpolSc1);
    } else {
#pragma unroll
        for (int k = 0; k < WPL; k += 2)
            __builtin_amdgcn_raw_buffer_store_b128((v4u32){v[k], tag, v[k + 1], tag}, rs, off + k * 8, 0, kCpolSc1);
    }
}
template <int WPL>
__device__ __forceinline__ Gran<WPL> gran_load(__amdgpu_buffer_rsrc_t rs, int off) {
    Gran<WPL> g;
    if constexpr (WPL == 1) {
        g.v[0] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, kCpolSc1);
    } else {
#pragma unroll
        for (int n = 0; n < WPL / 2; ++n) g.v[n] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + n * 16, 0, kCpolSc1);
    }
    return g;
}
template <int WPL>
__device__ __forceinline__ bool gran_ok(const Gran<WPL> &g, uint32_t want) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < WPL; ++k) ok = ok && g.tag(k) == want;
    return __all(ok);
}

template <int WPL>
__global__ __launch_bounds__(kPipeWaves * 64) void gol_lds_pipe_kernel(PipeArgs p) {
    constexpr int S = kPipeWaves;
    extern __shared__ uint4 pipe_smem[];
    const int Ww = p.Ww;  // == 64 * WPL (host-checked)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = p.nb, H = p.rows, T = p.turns;
    const int b = (p.xcd && nb % 8 == 0) ? (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    const int r0 = (int)((int64_t)b * H / nb);
    const int h = (int)((int64_t)(b + 1) * H / nb) - r0;
    const int bn = b + 1 == nb ? 0 : b + 1;
    // LDS: ring k < S - 1 = kPipeK row slots from slot k kPipeK; ring S - 1 =
    // p.kw slots after them; then one tag per slot; CONS[S]; 64 dummy words
    const int nslots = pipe_slots(p.kw);
    uint32_t *const R = reinterpret_cast<uint32_t *>(pipe_smem);
    lds_word *const TAG = (lds_word *)(R + (size_t)nslots * Ww);
    lds_word *const CONS = TAG + nslots;
    lds_word *const DUMMY = CONS + S;
    for (int i = threadIdx.x; i < nslots; i += blockDim.x) lds_put(TAG + i, 0);
    if (threadIdx.x < S) lds_put(CONS + threadIdx.x, 0);
    // generation 0: board rows [r0, r0 + h) into the last ring's slots 0 .. h - 1
    {
        const int base = (S - 1) * kPipeK, q4 = Ww / 4;
        for (int i = threadIdx.x; i < h * q4; i += blockDim.x) {
            const int r = i / q4, c = i - r * q4;
            const int br = r0 + r >= H ? r0 + r - H : r0 + r;
            reinterpret_cast<uint4 *>(R + (size_t)(base + r) * Ww)[c] =
                reinterpret_cast<const uint4 *>(p.src + (size_t)br * Ww)[c];
        }
    }
    const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
        p.edge, (short)0, (int)(pipe_edge_words(nb, Ww) * 4), 0x00020000);
    // this band's generation-0 rows 0 and 1 as the "turn 0" edges (slot 0) the
    // band above imports for turn 1 (waves 0 and 1, one row each)
    if (w < 2) {
        uint32_t v[WPL];
        const int br = r0 + w >= H ? r0 + w - H : r0 + w;
        lanes_load<WPL>(p.src + (size_t)br * Ww + lane * WPL, v);
        gran_store<WPL>(ers, (((b * kPipeQ + 0) * 2 + w) * 64 + lane) * WPL * 8, v, p.tag_base);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < h; i += blockDim.x) lds_put(TAG + (S - 1) * kPipeK + i, i + 1);
    __syncthreads();
    const int rin = w == 0 ? S - 1 : w - 1;  // the ring this wave reads
    const int in0 = rin * kPipeK, inm = rin == S - 1 ? p.kw - 1 : kPipeK - 1;
    const int out0 = w * kPipeK, outm = w == S - 1 ? p.kw - 1 : kPipeK - 1;
    const int loff = lane * WPL;             // the lane's first word of a row
    int in_seq = 0;                          // rows of ring rin read before this turn
    int out_seq = w == S - 1 ? h : 0;        // next row of ring w
    uint32_t cons_seen = 0;                  // CONS[w] as last read
    uint32_t econs_seen = 0, econs_val = 0;  // econs[b] as last read / in flight
    bool bail = false;
    uint32_t cnt = 0;
    long long tw[4] = {0, 0, 0, 0}, tf[3] = {0, 0, 0};
    const long long t_beg = (long long)__builtin_amdgcn_s_memrealtime();
    // A one-word signal (tag, CONS) written by lane 0; the other lanes write
    // dummy words of their own (no exec branch, no 64 stores to one address)
    auto signal = [&](lds_word *a, uint32_t v) __attribute__((always_inline)) {
        lds_put(lane == 0 ? a : DUMMY + lane, v);
    };
    // One poll of a bounded wait begun at t0, `spin` polls in: a short sleep
    // between polls; the global error word and the clock are consulted only
    // every 32nd poll (an L2 round trip costs about a microsecond).
    auto poll_ok = [&](long long t0, int spin) __attribute__((always_inline)) -> bool {
        if ((spin & 31) == 31) {
            if (__hip_atomic_load(p.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
                if (lane == 0) atomicOr(p.error, 1u);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
        return true;
    };
    auto lap = [&](int k, long long t0) __attribute__((always_inline)) {
        if (p.trace) tw[k] += (long long)__builtin_amdgcn_s_memrealtime() - t0;
    };

    for (int t = w + 1; t <= T && !bail; t += S) {
        const bool last = t == T;
        const int gT = (int)(((int64_t)r0 + T) % H);  // board row of the last turn's local row 0
        // econs[b], read one turn of this wave ahead of its use (every turn:
        // a conditional load made the compiler wait for it at once)
        if (econs_val > econs_seen) econs_seen = econs_val;
        econs_val = __hip_atomic_load(&p.econs[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // generation t - 1's ring row j (with its tag; settle() checks it)
        auto ring_issue = [&](int j) __attribute__((always_inline)) -> PipeRaw<WPL> {
            const int slot = in0 + ((in_seq + j) & inm);
            PipeRaw<WPL> r;
            r.tag = lds_get(TAG + slot);
            GOL_CBAR();
            lanes_load<WPL>(R + (size_t)slot * Ww + loff, r.w);
            return r;
        };
        auto settle = [&](int j, PipeRaw<WPL> x) __attribute__((always_inline)) -> PipeRaw<WPL> {
            const uint32_t want = (uint32_t)(in_seq + j + 1);
            if (__builtin_amdgcn_readfirstlane(x.tag) == want) return x;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            for (int spin = 0;; ++spin) {
                if (!poll_ok(t0, spin)) {
                    bail = true;
                    break;
                }
                x = ring_issue(j);
                if (__builtin_amdgcn_readfirstlane(x.tag) == want) break;
            }
            lap(0, t0);
            return x;
        };
        // Rows h, h + 1 of generation t - 1: the band below's first two (tagged
        // granules of edge slot (bn, (t - 1) % Q), tag base + t - 1; for t == 1
        // the slot 0 every band fills with its generation-0 rows at the start).
        // Issued once (mid-turn), checked at row h - 3.
        const uint32_t want_imp = p.tag_base + (uint32_t)(t - 1);
        const int eoff_in = ((bn * kPipeQ + (t - 1) % kPipeQ) * 2 * 64 + lane) * WPL * 8;
        struct Two {
            Gran<WPL> a, b;
        };
        auto imp_load = [&]() __attribute__((always_inline)) -> Two {
            Two r;
            r.a = gran_load<WPL>(ers, eoff_in);
            r.b = gran_load<WPL>(ers, eoff_in + 64 * WPL * 8);
            return r;
        };
        // (the slow path polls into temporaries and then reloads once: a
        // struct carried through the poll loop was kept in scratch)
        auto imp_settle = [&](const Two &r) __attribute__((always_inline)) -> bool {
            if (gran_ok<WPL>(r.a, want_imp) && gran_ok<WPL>(r.b, want_imp)) return true;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            for (int spin = 31;; spin += 32) {  // (every poll is an L2 round trip)
                if (!poll_ok(t0, spin)) {
                    bail = true;
                    break;
                }
                const Gran<WPL> a = gran_load<WPL>(ers, eoff_in), c = gran_load<WPL>(ers, eoff_in + 64 * WPL * 8);
                if (gran_ok<WPL>(a, want_imp) && gran_ok<WPL>(c, want_imp)) break;
            }
            lap(2, t0);
            return false;
        };
        // our rows 0 and 1 go to edge slot (b, t % Q) for the band above; the
        // slot must have been read (econs[b] >= t - Q)
        const int eoff_out = ((b * kPipeQ + t % kPipeQ) * 2 * 64 + lane) * WPL * 8;
        auto export_row = [&](int i, const uint32_t (&out)[WPL]) __attribute__((always_inline)) {
            // (econs[b] counts the turns of our edges the band above has read: turn
            // t - Q, the slot's last occupant, must be among them)
            if (i == 0 && t - kPipeQ + 1 > (int)econs_seen) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                for (int spin = 31; t - kPipeQ + 1 > (int)econs_seen; spin += 32) {
                    if (!poll_ok(t0, spin)) {
                        bail = true;
                        break;
                    }
                    econs_seen = __hip_atomic_load(&p.econs[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                lap(3, t0);
            }
            gran_store<WPL>(ers, eoff_out + i * 64 * WPL * 8, out, p.tag_base + (uint32_t)t);
        };
        // ring w: room for rows out_seq .. out_seq + n - 1
        auto room = [&](int n, uint32_t cn) __attribute__((always_inline)) {
            if (cn > cons_seen) cons_seen = cn;
            if (out_seq + n - 1 - (int)cons_seen <= outm) return;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            for (int spin = 0; out_seq + n - 1 - (int)cons_seen > outm; ++spin) {
                if (!poll_ok(t0, spin)) {
                    bail = true;
                    break;
                }
                cons_seen = lds_get(CONS + w);
            }
            lap(1, t0);
        };
        auto put = [&](const uint32_t (&out)[WPL]) __attribute__((always_inline)) {
            const int slot = out0 + (out_seq & outm);
            lanes_store<WPL>(R + (size_t)slot * Ww + loff, out);
            GOL_CBAR();
            signal(TAG + slot, (uint32_t)(out_seq + 1));
            ++out_seq;
        };
        auto emit_last = [&](int i, const uint32_t (&out)[WPL]) __attribute__((always_inline)) {
            const int g = gT + i >= H ? gT + i - H : gT + i;
            lanes_store<WPL>(p.dst + (size_t)g * Ww + loff, out);
#pragma unroll
            for (int k = 0; k < WPL; ++k) cnt += __builtin_popcount(out[k]);
        };

        LdsRow<WPL> s[3];
        PipeRaw<WPL> x[3];
        Two imp;
        auto rule = [&](int q, int qb, int qn, uint32_t (&out)[WPL]) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < WPL; ++k)
                out[k] = rule_word(s[q].s0[k], s[q].s1[k], s[qb].s0[k], s[qb].s1[k], s[qn].s0[k], s[qn].s1[k],
                                   s[qb].c[k]);
        };
        // Generic row i (the first three and the last rows of a turn): row i + 3
        // may be an import; rows 0, 1 are exported.
        auto row = [&](auto qc, auto lastc, int i) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value, qb = (q + 1) % 3, qn = (q + 2) % 3;
            constexpr bool LAST = decltype(lastc)::value;
            if (i + 2 < h) {
                x[q] = settle(i + 2, x[q]);
                signal(CONS + rin, (uint32_t)(in_seq + i + 3));  // rows read so far
            }
            if (i + 3 < h) {
                x[qb] = ring_issue(i + 3);
            } else if (i + 3 <= h + 1) {
                if (i + 3 == h && !imp_settle(imp)) imp = imp_load();  // (now complete: reload)
                // row h or h + 1, picked with a mask: a select of the two (or a
                // reference) became a load through a selected pointer, which
                // kept the import rows in scratch
                const uint32_t m = i + 3 == h ? ~0u : 0u;
#pragma unroll
                for (int k = 0; k < WPL; ++k) x[qb].w[k] = (imp.a.word(k) & m) | (imp.b.word(k) & ~m);
            }
            const uint32_t cn = LAST ? 0u : lds_get(CONS + w);
            pipe_sums<WPL>(x[q].w, s[qn]);
            uint32_t out[WPL];
            rule(q, qb, qn, out);
            if constexpr (LAST) {
                emit_last(i, out);
            } else {
                if (i < 2) export_row(i, out);
                room(1, cn);
                put(out);
            }
        };
        // Steady rows (3 <= i, i + 5 < h): every input row from the ring, no
        // export; CONS published and ring room checked once a group of three
        // (with a CONS value read during the previous group).
        uint32_t cons_next = 0;
        auto frow = [&](auto qc, auto lastc, int i) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value, qb = (q + 1) % 3, qn = (q + 2) % 3;
            constexpr bool LAST = decltype(lastc)::value;
            x[q] = settle(i + 2, x[q]);
            if constexpr (q == 2) signal(CONS + rin, (uint32_t)(in_seq + i + 3));
            x[qb] = ring_issue(i + 3);
            if constexpr (!LAST && q == 1) cons_next = lds_get(CONS + w);
            pipe_sums<WPL>(x[q].w, s[qn]);
            uint32_t out[WPL];
            rule(q, qb, qn, out);
            if constexpr (LAST) {
                emit_last(i, out);
            } else {
                if constexpr (q == 0) room(3, cons_next);
                put(out);
            }
        };
        auto fast = [&](auto lastc, int i0, int i1) __attribute__((always_inline)) {
            const long long f0 = p.trace ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
            const long long w0 = tw[0];
            for (int i = i0; i < i1; i += 3) {
                frow(std::integral_constant<int, 0>{}, lastc, i);
                frow(std::integral_constant<int, 1>{}, lastc, i + 1);
                frow(std::integral_constant<int, 2>{}, lastc, i + 2);
            }
            if (p.trace) {  // steady-state rows: ticks, rows, ring-row waits among them
                tf[0] += (long long)__builtin_amdgcn_s_memrealtime() - f0;
                tf[1] += i1 > i0 ? i1 - i0 : 0;
                tf[2] += tw[0] - w0;
            }
        };
        // rows 3 .. fe - 1 run steady (fe: the largest 3 + 3k with fe + 3 <= h - 2);
        // the imports are issued at row fm (the middle) and checked at row h - 3
        const int fe = h >= 9 ? 3 + 3 * ((h - 8) / 3) : 0;
        const int fm = h >= 9 ? 3 + 3 * ((fe - 3) / 6) : 0;
        auto rows = [&](auto lastc) __attribute__((always_inline)) {
            x[1] = ring_issue(0);
            if (h > 1) x[2] = ring_issue(1);
            if (fe == 0) imp = imp_load();  // (short bands: at once)
            if (h > 2) x[0] = ring_issue(2);
            x[1] = settle(0, x[1]);
            x[2] = settle(1, x[2]);
            if (h == 2) {  // row 2 is the first import
                if (!imp_settle(imp)) imp = imp_load();
#pragma unroll
                for (int k = 0; k < WPL; ++k) x[0].w[k] = imp.a.word(k);
            }
            pipe_sums<WPL>(x[1].w, s[0]);
            pipe_sums<WPL>(x[2].w, s[1]);
            int i = 0;
            if (fe > 0) {
                row(std::integral_constant<int, 0>{}, lastc, 0);
                row(std::integral_constant<int, 1>{}, lastc, 1);
                row(std::integral_constant<int, 2>{}, lastc, 2);
                cons_next = cons_seen;
                fast(lastc, 3, fm);
                imp = imp_load();
                fast(lastc, fm, fe);
                i = fe;
            }
            for (; i + 3 <= h && !bail; i += 3) {
                row(std::integral_constant<int, 0>{}, lastc, i);
                row(std::integral_constant<int, 1>{}, lastc, i + 1);
                row(std::integral_constant<int, 2>{}, lastc, i + 2);
            }
            if (i < h && !bail) row(std::integral_constant<int, 0>{}, lastc, i);
            if (i + 1 < h && !bail) row(std::integral_constant<int, 1>{}, lastc, i + 1);
        };
        if (last)
            rows(std::true_type{});
        else
            rows(std::false_type{});
        in_seq += h;
        signal(CONS + rin, (uint32_t)in_seq);  // (h == 2: the rows loop counts no row)
        // generation t - 1's edges of the band below are in registers: turns
        // 0 .. t - 1 of its edges read
        if (lane == 0) __hip_atomic_store(&p.econs[bn], (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p.trace && lane == 0) {
        for (int k = 0; k < 4; ++k) atomicAdd(&p.trace[k], (unsigned long long)tw[k]);
        atomicAdd(&p.trace[4], (unsigned long long)((long long)__builtin_amdgcn_s_memrealtime() - t_beg));
        for (int k = 0; k < 3; ++k) atomicAdd(&p.trace[8 + k], (unsigned long long)tf[k]);
    }
    if (p.alive) {
        const uint32_t tot = wave_sum_u32(cnt);
        if (lane == 0 && tot) atomicAdd(p.alive, (unsigned long long)tot);
    }
}
#undef GOL_CBAR

template <typename F>
static hipError_t dispatch_pipe(int wpl, F &&f) {
    if (wpl == 1) return f(gol_lds_pipe_kernel<1>);
    if (wpl == 2) return f(gol_lds_pipe_kernel<2>);
    if (wpl == 4) return f(gol_lds_pipe_kernel<4>);
    return hipErrorInvalidValue;
}
int pipe_blocks_per_cu(int wpl, int64_t lds_bytes) {
    int n = 0;
    hipError_t e = dispatch_pipe(wpl, [&](auto kern) {
        hipError_t r = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        return r == hipSuccess ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, kPipeWaves * 64, (size_t)lds_bytes)
                               : r;
    });
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}
hipError_t launch_pipe(const PipeArgs &p, int wpl, hipStream_t s) {
    if (p.Ww != 64 * wpl || p.nb < 1 || p.kw < p.hmax + 4 || (p.kw & (p.kw - 1))) return hipErrorInvalidValue;
    const size_t bytes = (size_t)pipe_lds_bytes(p.Ww, p.kw);
    return dispatch_pipe(wpl, [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(p.nb), dim3(kPipeWaves * 64), bytes, s, p);
        return hipGetLastError();
    });
}

}  // namespace golk
