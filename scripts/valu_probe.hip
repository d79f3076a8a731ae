// VALU issue-rate probe for the step kernel's instruction mix on gfx950.
// Each variant runs a fixed block of 16 instructions (inline asm, registers
// chosen by hand) in a loop; reported as wave-instructions per SIMD per cycle
// at the measured rate over 256 CUs x 4 SIMDs x 2.4 GHz.  No memory traffic.
//   hipcc -O3 --offload-arch=gfx950 -o valu_probe scripts/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define B3(d, a, b, c) "v_bitop3_b32 v" #d ", v" #a ", v" #b ", v" #c " bitop3:0x96\n"
#define DPP(d, a) "v_mov_b32_dpp v" #d ", v" #a " wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define ALB(d, a, b) "v_alignbit_b32 v" #d ", v" #a ", v" #b ", 31\n"

// 16 independent bitop3, three sources in three banks
#define V_INDEP B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) \
                B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49)
// 16 independent bitop3, three sources in one bank
#define V_BANK3 B3(40,48,52,56) B3(41,49,53,57) B3(42,50,54,58) B3(43,51,55,59) B3(44,52,56,60) B3(45,53,57,61) B3(46,54,58,62) B3(47,55,59,63) \
                B3(40,48,52,56) B3(41,49,53,57) B3(42,50,54,58) B3(43,51,55,59) B3(44,52,56,60) B3(45,53,57,61) B3(46,54,58,62) B3(47,55,59,63)
// two sources in one bank
#define V_BANK2 B3(40,48,52,49) B3(41,49,53,50) B3(42,50,54,51) B3(43,51,55,52) B3(44,52,56,53) B3(45,53,57,54) B3(46,54,58,55) B3(47,55,59,56) \
                B3(40,48,52,49) B3(41,49,53,50) B3(42,50,54,51) B3(43,51,55,52) B3(44,52,56,53) B3(45,53,57,54) B3(46,54,58,55) B3(47,55,59,56)
// one chain: each reads the previous result
#define V_CHAIN1 B3(40,40,49,50) B3(40,40,50,51) B3(40,40,51,52) B3(40,40,52,53) B3(40,40,53,54) B3(40,40,54,55) B3(40,40,55,56) B3(40,40,56,57) \
                 B3(40,40,57,58) B3(40,40,58,59) B3(40,40,59,60) B3(40,40,60,61) B3(40,40,61,62) B3(40,40,62,63) B3(40,40,63,49) B3(40,40,49,50)
// two interleaved chains
#define V_CHAIN2 B3(40,40,49,50) B3(41,41,50,51) B3(40,40,51,52) B3(41,41,52,53) B3(40,40,53,54) B3(41,41,54,55) B3(40,40,55,56) B3(41,41,56,57) \
                 B3(40,40,57,58) B3(41,41,58,59) B3(40,40,59,60) B3(41,41,60,61) B3(40,40,61,62) B3(41,41,62,63) B3(40,40,63,49) B3(41,41,49,50)
// four interleaved chains
#define V_CHAIN4 B3(40,40,49,50) B3(41,41,50,51) B3(42,42,51,52) B3(43,43,52,53) B3(40,40,53,54) B3(41,41,54,55) B3(42,42,55,56) B3(43,43,56,57) \
                 B3(40,40,57,58) B3(41,41,58,59) B3(42,42,59,60) B3(43,43,60,61) B3(40,40,61,62) B3(41,41,62,63) B3(42,42,63,49) B3(43,43,49,50)
#define V_DPP DPP(40,48) DPP(41,49) DPP(42,50) DPP(43,51) DPP(44,52) DPP(45,53) DPP(46,54) DPP(47,55) \
              DPP(40,56) DPP(41,57) DPP(42,58) DPP(43,59) DPP(44,60) DPP(45,61) DPP(46,62) DPP(47,63)
#define V_ALB ALB(40,48,49) ALB(41,49,50) ALB(42,50,51) ALB(43,51,52) ALB(44,52,53) ALB(45,53,54) ALB(46,54,55) ALB(47,55,56) \
              ALB(40,56,57) ALB(41,57,58) ALB(42,58,59) ALB(43,59,60) ALB(44,60,61) ALB(45,61,62) ALB(46,62,63) ALB(47,63,48)
// 12 bitop3 : 2 dpp : 2 alignbit = 6 : 1 : 1 (16 instructions; named "mix9:1:1" before round 5, which it is not)
#define V_MIX B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) DPP(43,60) B3(44,52,53,54) B3(45,53,54,55) ALB(46,61,62) B3(47,55,56,57) \
              B3(40,56,57,58) B3(41,57,58,59) DPP(42,63) B3(43,59,60,61) B3(44,60,61,62) ALB(45,61,48) B3(46,62,63,48) B3(47,63,48,49)

// the step kernels' ratio per word-turn at two words per lane, 9 bitop3 : 1 dpp : 1 alignbit
// (22 = 18 + 2 + 2), independent, the shifts spread over the block
#define V_MIX911 B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) DPP(44,60) B3(45,53,54,55) B3(46,54,55,56) \
                 B3(47,55,56,57) B3(40,56,57,58) B3(41,57,58,59) ALB(42,61,62) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) \
                 B3(46,62,63,48) DPP(47,63) B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) ALB(43,62,48) B3(44,52,53,54) B3(45,53,54,55)
// 10 : 1 : 1 per word at four words per lane (quads: 1/2 DPP + 1/2 alignbit per word): 20 + 1 + 1 = 22
#define V_MIX10 B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) DPP(45,60) B3(46,54,55,56) \
                B3(47,55,56,57) B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) \
                B3(46,62,63,48) B3(47,63,48,49) ALB(40,61,62) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(46,53,54,55)
// 15 bitop3 + 1 dpp / 1 alignbit; 12 + 4 spread; 12 + 4 grouped
#define V_D1 B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) DPP(47,60) \
             B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49)
#define V_A1 B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) ALB(47,60,61) \
             B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49)
#define V_D4S B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) DPP(43,60) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) DPP(47,61) \
              B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) DPP(43,62) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) DPP(47,63)
#define V_A4S B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) ALB(43,60,61) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) ALB(47,61,62) \
              B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) ALB(43,62,63) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) ALB(47,63,48)
#define V_D4G B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) \
              B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) DPP(43,60) DPP(47,61) DPP(43,62) DPP(47,63)
#define V_A4G B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) \
              B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) ALB(43,60,61) ALB(47,61,62) ALB(43,62,63) ALB(47,63,48)
// VALU that is not bitop3: v_xor_b32 (VOP2) and v_and_or (VOP3), independent
#define XOR(d, a, b) "v_xor_b32 v" #d ", v" #a ", v" #b "\n"
#define V_XOR XOR(40,48,49) XOR(41,49,50) XOR(42,50,51) XOR(43,51,52) XOR(44,52,53) XOR(45,53,54) XOR(46,54,55) XOR(47,55,56) \
              XOR(40,56,57) XOR(41,57,58) XOR(42,58,59) XOR(43,59,60) XOR(44,60,61) XOR(45,61,62) XOR(46,62,63) XOR(47,63,48)

// Lane 0 of each workgroup records the shader-clock and the constant-rate
// (100 MHz) counter around its loop, so the rate is also reported per cycle
// of the clock the CU actually ran at.
constexpr int nlines(const char* t) { int n = 0; for (; *t; ++t) n += *t == '\n'; return n; }
#define KERNEL(name, body)                                                        \
    constexpr int name##_n = nlines(body);                                        \
    __global__ void name(int iters, long long* sink) {                           \
        const long long c0 = clock64(), w0 = wall_clock64();                      \
        for (int i = 0; i < iters; ++i) asm volatile(".rept 16\n" body ".endr\n" ::: CLOB); \
        const long long c1 = clock64(), w1 = wall_clock64();                      \
        if (threadIdx.x == 0) { sink[2 * blockIdx.x] = c1 - c0; sink[2 * blockIdx.x + 1] = w1 - w0; } \
    }
KERNEL(k_indep, V_INDEP)
KERNEL(k_bank3, V_BANK3)
KERNEL(k_bank2, V_BANK2)
KERNEL(k_chain1, V_CHAIN1)
KERNEL(k_chain2, V_CHAIN2)
KERNEL(k_chain4, V_CHAIN4)
KERNEL(k_dpp, V_DPP)
KERNEL(k_alb, V_ALB)
KERNEL(k_mix, V_MIX)
KERNEL(k_mix911, V_MIX911)
KERNEL(k_mix10, V_MIX10)
KERNEL(k_d1, V_D1)
KERNEL(k_a1, V_A1)
KERNEL(k_d4s, V_D4S)
KERNEL(k_a4s, V_A4S)
KERNEL(k_d4g, V_D4G)
KERNEL(k_a4g, V_A4G)
KERNEL(k_xor, V_XOR)

#define P_real_HHHVVH DPP(40,60) ALB(41,61,49) DPP(42,62) B3(40,48,49,50) B3(41,49,50,51) ALB(45,63,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) B3(40,56,57,58) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49) B3(40,48,49,50) B3(41,49,50,51)
KERNEL(k_real_HHHVVH, P_real_HHHVVH)
#define P_real_spread DPP(40,60) B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) ALB(45,61,49) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) B3(40,56,57,58) DPP(43,62) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) ALB(41,63,51) B3(46,62,63,48) B3(47,63,48,49) B3(40,48,49,50) B3(41,49,50,51)
KERNEL(k_real_spread, P_real_spread)
#define P_HH_pairs DPP(40,60) ALB(41,61,49) B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) B3(40,56,57,58) DPP(43,62) ALB(44,63,51) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49) B3(40,48,49,50) B3(41,49,50,51)
KERNEL(k_HH_pairs, P_HH_pairs)
#define P_HV_alt DPP(40,60) B3(40,48,49,50) ALB(42,61,49) B3(41,49,50,51) DPP(44,62) B3(42,50,51,52) ALB(46,63,51) B3(43,51,52,53) DPP(40,60) B3(44,52,53,54) ALB(42,61,49) B3(45,53,54,55) DPP(44,62) B3(46,54,55,56) ALB(46,63,51) B3(47,55,56,57) DPP(40,60) B3(40,56,57,58) ALB(42,61,49) B3(41,57,58,59) DPP(44,62) B3(42,58,59,60)
KERNEL(k_HV_alt, P_HV_alt)
#define P_HVV DPP(40,60) B3(40,48,49,50) B3(41,49,50,51) ALB(43,61,49) B3(42,50,51,52) B3(43,51,52,53) DPP(46,62) B3(44,52,53,54) B3(45,53,54,55) ALB(41,63,51) B3(46,54,55,56) B3(47,55,56,57) DPP(44,60) B3(40,56,57,58) B3(41,57,58,59) ALB(47,61,49) B3(42,58,59,60) B3(43,59,60,61) DPP(42,62) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48)
KERNEL(k_HVV, P_HVV)
#define P_HVVV DPP(40,60) B3(40,48,49,50) B3(41,49,50,51) B3(42,50,51,52) ALB(44,61,49) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) DPP(40,62) B3(46,54,55,56) B3(47,55,56,57) B3(40,56,57,58) ALB(44,63,51) B3(41,57,58,59) B3(42,58,59,60) B3(43,59,60,61) DPP(40,60) B3(44,60,61,62) B3(45,61,62,63) B3(46,62,63,48) B3(47,63,48,49) B3(40,48,49,50)
KERNEL(k_HVVV, P_HVVV)
// LDS-crossbar lane exchange instead of DPP: ds_bpermute (no LDS memory),
// one in flight per 16-instruction block (lgkmcnt(1)), two in flight (2)
#define BP(d, a, b) "ds_bpermute_b32 v" #d ", v" #a ", v" #b "\n"
#define P_bperm_alb BP(41,62,63) B3(40,48,49,50) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) ALB(40,60,61) \
              B3(42,56,57,58) B3(43,57,58,59) B3(44,58,59,60) B3(45,59,60,61) B3(46,60,61,62) B3(47,61,62,63) B3(40,62,63,48) "s_waitcnt lgkmcnt(1)\n"
#define P_bperm2_alb2 BP(41,62,63) B3(40,48,49,50) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) ALB(45,53,54) B3(46,54,55,56) B3(47,55,56,57) BP(43,60,61) \
              B3(42,56,57,58) B3(40,57,58,59) B3(44,58,59,60) ALB(45,59,60) B3(46,60,61,62) B3(47,61,62,63) B3(40,62,63,48) "s_waitcnt lgkmcnt(2)\n"
#define P_dpp_alb DPP(41,62) B3(40,48,49,50) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) B3(45,53,54,55) B3(46,54,55,56) B3(47,55,56,57) ALB(40,60,61) \
              B3(42,56,57,58) B3(43,57,58,59) B3(44,58,59,60) B3(45,59,60,61) B3(46,60,61,62) B3(47,61,62,63) B3(40,62,63,48) "s_nop 0\n"
#define P_dpp2_alb2 DPP(41,62) B3(40,48,49,50) B3(42,50,51,52) B3(43,51,52,53) B3(44,52,53,54) ALB(45,53,54) B3(46,54,55,56) B3(47,55,56,57) DPP(43,60) \
              B3(42,56,57,58) B3(40,57,58,59) B3(44,58,59,60) ALB(45,59,60) B3(46,60,61,62) B3(47,61,62,63) B3(40,62,63,48) "s_nop 0\n"
#define P_xor_e64 "v_xor_b32_e64 v40, v48, v49\nv_xor_b32_e64 v41, v49, v50\nv_xor_b32_e64 v42, v50, v51\nv_xor_b32_e64 v43, v51, v52\n"
#define P_andor "v_and_or_b32 v40, v48, v49, v50\nv_and_or_b32 v41, v49, v50, v51\nv_and_or_b32 v42, v50, v51, v52\nv_and_or_b32 v43, v51, v52, v53\n"
KERNEL(k_bperm_alb, P_bperm_alb)
KERNEL(k_bperm2_alb2, P_bperm2_alb2)
KERNEL(k_dpp_alb, P_dpp_alb)
KERNEL(k_dpp2_alb2, P_dpp2_alb2)
KERNEL(k_xor_e64, P_xor_e64)
KERNEL(k_xor3, P_andor)

typedef void (*kfn)(int, long long*);

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    long long* sink;
    CK(hipMalloc(&sink, 16 * cus));
    long long* hs = (long long*)malloc(16 * cus);
    struct { const char* n; kfn f; int len; } ks[] = {{"indep", k_indep, k_indep_n}, {"bank3", k_bank3, k_bank3_n}, {"bank2", k_bank2, k_bank2_n},
        {"chain1", k_chain1, k_chain1_n}, {"chain2", k_chain2, k_chain2_n}, {"chain4", k_chain4, k_chain4_n}, {"dpp", k_dpp, k_dpp_n}, {"alignbit", k_alb, k_alb_n}, {"mix6:1:1", k_mix, k_mix_n}, {"mix9:1:1", k_mix911, k_mix911_n}, {"mix10:1:1", k_mix10, k_mix10_n},
        {"b3x15+dpp", k_d1, k_d1_n}, {"b3x15+alb", k_a1, k_a1_n}, {"b3x12+dpp4spread", k_d4s, k_d4s_n}, {"b3x12+alb4spread", k_a4s, k_a4s_n}, {"b3x12+dpp4grouped", k_d4g, k_d4g_n},
        {"b3x12+alb4grouped", k_a4g, k_a4g_n}, {"xor_vop2", k_xor, k_xor_n}, {"real_HHHVVH", k_real_HHHVVH, k_real_HHHVVH_n}, {"real_spread", k_real_spread, k_real_spread_n}, {"HH_pairs", k_HH_pairs, k_HH_pairs_n}, {"HV_alt", k_HV_alt, k_HV_alt_n}, {"HVV", k_HVV, k_HVV_n}, {"HVVV", k_HVVV, k_HVVV_n}, {"bperm_alb", k_bperm_alb, k_bperm_alb_n}, {"bperm2_alb2", k_bperm2_alb2, k_bperm2_alb2_n}, {"dpp_alb", k_dpp_alb, k_dpp_alb_n}, {"dpp2_alb2", k_dpp2_alb2, k_dpp2_alb2_n}, {"xor_e64", k_xor_e64, k_xor_e64_n}, {"xor3", k_xor3, k_xor3_n}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int wps : {1, 2, 4}) {
        for (auto& k : ks) {
            const int threads = 64 * 4 * wps;  // wps waves per SIMD, one workgroup per CU
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, 10, sink);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, iters, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double winst = double(cus) * 4 * wps * iters * 16 * k.len;  // wave-instructions
            const double per_simd_cycle = winst / (ms * 1e-3) / (cus * 4.0 * 2.4e9);
            CK(hipMemcpy(hs, sink, 16 * cus, hipMemcpyDeviceToHost));
            double cyc = 0, wall = 0;
            for (int b = 0; b < cus; ++b) cyc += hs[2 * b], wall += hs[2 * b + 1];
            const double ghz = cyc / (wall / 100e6) / 1e9;  // shader clock over the 100 MHz counter
            // per SIMD and per cycle of the clock the CUs ran at: the measured
            // clock x the event-timed wall time (round 5; before, the in-kernel
            // cycle sum of lane 0 alone, which under-counted: values > 0.5)
            const double per_cycle = winst / (ms * 1e-3) / (cus * 4.0 * ghz * 1e9);
            printf("{\"variant\": \"%s\", \"len\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
                   "\"winst_per_simd_cycle_2p4\": %.4f, \"clock_ghz\": %.3f, \"winst_per_simd_cycle\": %.4f}\n",
                   k.n, k.len, wps, ms, per_simd_cycle, ghz, per_cycle);
        }
    }
    return 0;
}
