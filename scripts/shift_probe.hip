// Issue-rate probe: horizontal one-cell shifts as DPP + alignbit (current
// step kernel) vs a lane-mask carry: v_cmp (sign bits -> SGPR lane mask),
// s_lshl_b64 (mask moves one lane, on the scalar unit), v_addc_co_u32
// (x + x + carry-in = x << 1 with the left lane's top bit).  Blocks model the
// per-word-turn mix of words-per-lane 1 / 2 / 4 (9 bitop3 per word-turn).
//   hipcc -O3 --offload-arch=gfx950 -o shift_probe scripts/shift_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", \
    "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "vcc", "scc"
#define B3(d, a, b, c) "v_bitop3_b32 v" #d ", v" #a ", v" #b ", v" #c " bitop3:0x96\n"
#define DPP(d, a) "v_mov_b32_dpp v" #d ", v" #a " wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define ALB(d, a, b) "v_alignbit_b32 v" #d ", v" #a ", v" #b ", 31\n"
#define CMPA(v) "v_cmp_gt_i32_e64 s[20:21], 0, v" #v "\n"
#define CMPB(v) "v_cmp_gt_i32_e64 s[22:23], 0, v" #v "\n"
#define SLA "s_lshl_b64 s[20:21], s[20:21], 1\n"
#define SLB "s_lshl_b64 s[22:23], s[22:23], 1\n"
#define ADA(d, v) "v_addc_co_u32_e64 v" #d ", s[24:25], v" #v ", v" #v ", s[20:21]\n"
#define ADB(d, v) "v_addc_co_u32_e64 v" #d ", s[26:27], v" #v ", v" #v ", s[22:23]\n"

#define B3x6a B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55)
#define B3x6b B3(46,54,55,56) B3(47,55,56,57) B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61)
#define B3x6c B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49) B3(40,48,50,52) B3(41,49,51,53)
// WPL 2: 18 bitop3 + two shifts (one pair-row: 2 words)
#define OLD2 DPP(44,60) DPP(45,61) B3x6a ALB(46,60,44) ALB(47,45,61) B3x6b B3x6c
#define NEW2 CMPA(60) CMPB(61) B3(40,48,49,50) B3(41,49,50,51) SLA SLB B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) \
    ADA(46,60) ADB(47,61) B3x6b B3x6c
// WPL 4: 36 bitop3 + two shifts (4 words)
#define OLD4 DPP(44,60) DPP(45,61) B3x6a ALB(46,60,44) ALB(47,45,61) B3x6b B3x6c B3x6a B3x6b B3x6c
#define NEW4 CMPA(60) CMPB(61) B3(40,48,49,50) B3(41,49,50,51) SLA SLB B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) \
    ADA(46,60) ADB(47,61) B3x6b B3x6c B3x6a B3x6b B3x6c
// WPL 1: 18 bitop3 + four shifts (2 words); new: two dependent shifts per word
#define OLD1 DPP(44,60) DPP(45,61) B3x6a ALB(46,60,44) ALB(47,45,61) DPP(44,62) DPP(45,63) B3x6b ALB(46,62,44) ALB(47,45,63) B3x6c
#define NEW1 CMPA(60) CMPB(61) B3(40,48,49,50) B3(41,49,50,51) SLA SLB B3(42,50,51,52) B3(43,51,52,53) ADA(46,60) ADB(47,61) \
    B3(44,52,53,54) B3(45,53,54,55) CMPA(46) CMPB(47) B3x6b SLA SLB ADA(44,46) ADB(45,47) B3x6c
#define BASE2 B3x6a B3x6b B3x6c

constexpr int nlines(const char* t) { int n = 0; for (; *t; ++t) n += *t == '\n'; return n; }
#define KERNEL(name, body)                                                        \
    constexpr int name##_n = nlines(body);                                        \
    __global__ void name(int iters, long long* sink) {                           \
        for (int i = 0; i < iters; ++i) asm volatile(".rept 16\n" body ".endr\n" ::: CLOB); \
        if (threadIdx.x == 0) sink[blockIdx.x] = iters;                          \
    }
KERNEL(k_old2, OLD2)
KERNEL(k_new2, NEW2)
KERNEL(k_old4, OLD4)
KERNEL(k_new4, NEW4)
KERNEL(k_old1, OLD1)
KERNEL(k_new1, NEW1)
KERNEL(k_base, BASE2)
typedef void (*kfn)(int, long long*);

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    long long* sink;
    CK(hipMalloc(&sink, 8 * cus));
    // words: word-turns per block (per lane)
    struct { const char* n; kfn f; int len; int words; } ks[] = {
        {"old_wpl2", k_old2, k_old2_n, 2}, {"new_wpl2", k_new2, k_new2_n, 2}, {"old_wpl4", k_old4, k_old4_n, 4},
        {"new_wpl4", k_new4, k_new4_n, 4}, {"old_wpl1", k_old1, k_old1_n, 2}, {"new_wpl1", k_new1, k_new1_n, 2},
        {"bitop3_only_18", k_base, k_base_n, 2}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int wps : {2, 3, 4}) {
        for (int rep = 0; rep < 2; ++rep)
        for (auto& k : ks) {
            const int threads = 64 * 4 * wps;
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, 10, sink);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, iters, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double winst = double(cus) * 4 * wps * iters * 16 * k.len;
            const double wordturns = double(cus) * 4 * wps * iters * 16 * k.words * 64;
            printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"rep\": %d, \"ms\": %.3f, \"winst_per_simd_cycle_2p4\": %.4f, "
                   "\"ns_per_Gwordturn\": %.4f, \"cell_updates_T_per_s\": %.1f}\n",
                   k.n, wps, rep, ms, winst / (ms * 1e-3) / (cus * 4.0 * 2.4e9), ms * 1e6 / (wordturns / 1e9),
                   wordturns * 32 / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
