// VGPR bank probe: does the operand register bank (vgpr index mod 4) change the issue cost
// of the ChaCha20 instruction mix on gfx950? Each kernel runs a fixed asm body on explicitly
// named VGPRs (v40..v63) many times, 8 waves per SIMD, and reports cycles per
// wave-instruction per SIMD at the measured shader clock (s_memtime, 100 MHz ref in
// s_memrealtime).
//   add_same / add_diff   v_add_u32 with both sources in one bank / in different banks
//   xor_same / xor_diff   the same for v_xor_b32
//   qr_col / qr_row       one ChaCha20 double round (8 quarter rounds, 96 ops) with the state
//                         word x[4r+c] in v[40 + 4c + r] (bank = r: no op reads two operands of
//                         one bank) or in v[40 + 4r + c] (bank = c: every column quarter round
//                         reads both operands from one bank)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench9 tools/microbench9.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <string>

#define STR_(x) #x
#define STR(x) STR_(x)

// 16 independent v_add_u32 per block
#define ADD_SAME                                                                                         \
  "v_add_u32 v40, v40, v44\n v_add_u32 v41, v41, v45\n v_add_u32 v42, v42, v46\n v_add_u32 v43, v43, v47\n" \
  "v_add_u32 v48, v48, v52\n v_add_u32 v49, v49, v53\n v_add_u32 v50, v50, v54\n v_add_u32 v51, v51, v55\n" \
  "v_add_u32 v44, v44, v56\n v_add_u32 v45, v45, v57\n v_add_u32 v46, v46, v58\n v_add_u32 v47, v47, v59\n" \
  "v_add_u32 v52, v52, v60\n v_add_u32 v53, v53, v61\n v_add_u32 v54, v54, v62\n v_add_u32 v55, v55, v63\n"
#define ADD_DIFF                                                                                         \
  "v_add_u32 v40, v40, v45\n v_add_u32 v41, v41, v46\n v_add_u32 v42, v42, v47\n v_add_u32 v43, v43, v44\n" \
  "v_add_u32 v48, v48, v53\n v_add_u32 v49, v49, v54\n v_add_u32 v50, v50, v55\n v_add_u32 v51, v51, v52\n" \
  "v_add_u32 v44, v44, v57\n v_add_u32 v45, v45, v58\n v_add_u32 v46, v46, v59\n v_add_u32 v47, v47, v56\n" \
  "v_add_u32 v52, v52, v61\n v_add_u32 v53, v53, v62\n v_add_u32 v54, v54, v63\n v_add_u32 v55, v55, v60\n"

// quarter round on named registers: a += b; d ^= a; d <<<= 16; c += d; b ^= c; b <<<= 12;
//                                   a += b; d ^= a; d <<<= 8;  c += d; b ^= c; b <<<= 7
#define QR(a, b, c, d)                                                                           \
  "v_add_u32 " a ", " a ", " b "\n v_xor_b32 " d ", " d ", " a "\n v_alignbit_b32 " d ", " d ", " d ", 16\n" \
  "v_add_u32 " c ", " c ", " d "\n v_xor_b32 " b ", " b ", " c "\n v_alignbit_b32 " b ", " b ", " b ", 20\n" \
  "v_add_u32 " a ", " a ", " b "\n v_xor_b32 " d ", " d ", " a "\n v_alignbit_b32 " d ", " d ", " d ", 24\n" \
  "v_add_u32 " c ", " c ", " d "\n v_xor_b32 " b ", " b ", " c "\n v_alignbit_b32 " b ", " b ", " b ", 25\n"

// interleave the 4 quarter rounds of a half round op by op (what the compiler schedules)
#define QR4(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3)                              \
  "v_add_u32 " a0 ", " a0 ", " b0 "\n v_add_u32 " a1 ", " a1 ", " b1 "\n v_add_u32 " a2 ", " a2 ", " b2 "\n v_add_u32 " a3 ", " a3 ", " b3 "\n" \
  "v_xor_b32 " d0 ", " d0 ", " a0 "\n v_xor_b32 " d1 ", " d1 ", " a1 "\n v_xor_b32 " d2 ", " d2 ", " a2 "\n v_xor_b32 " d3 ", " d3 ", " a3 "\n" \
  "v_alignbit_b32 " d0 ", " d0 ", " d0 ", 16\n v_alignbit_b32 " d1 ", " d1 ", " d1 ", 16\n v_alignbit_b32 " d2 ", " d2 ", " d2 ", 16\n v_alignbit_b32 " d3 ", " d3 ", " d3 ", 16\n" \
  "v_add_u32 " c0 ", " c0 ", " d0 "\n v_add_u32 " c1 ", " c1 ", " d1 "\n v_add_u32 " c2 ", " c2 ", " d2 "\n v_add_u32 " c3 ", " c3 ", " d3 "\n" \
  "v_xor_b32 " b0 ", " b0 ", " c0 "\n v_xor_b32 " b1 ", " b1 ", " c1 "\n v_xor_b32 " b2 ", " b2 ", " c2 "\n v_xor_b32 " b3 ", " b3 ", " c3 "\n" \
  "v_alignbit_b32 " b0 ", " b0 ", " b0 ", 20\n v_alignbit_b32 " b1 ", " b1 ", " b1 ", 20\n v_alignbit_b32 " b2 ", " b2 ", " b2 ", 20\n v_alignbit_b32 " b3 ", " b3 ", " b3 ", 20\n" \
  "v_add_u32 " a0 ", " a0 ", " b0 "\n v_add_u32 " a1 ", " a1 ", " b1 "\n v_add_u32 " a2 ", " a2 ", " b2 "\n v_add_u32 " a3 ", " a3 ", " b3 "\n" \
  "v_xor_b32 " d0 ", " d0 ", " a0 "\n v_xor_b32 " d1 ", " d1 ", " a1 "\n v_xor_b32 " d2 ", " d2 ", " a2 "\n v_xor_b32 " d3 ", " d3 ", " a3 "\n" \
  "v_alignbit_b32 " d0 ", " d0 ", " d0 ", 24\n v_alignbit_b32 " d1 ", " d1 ", " d1 ", 24\n v_alignbit_b32 " d2 ", " d2 ", " d2 ", 24\n v_alignbit_b32 " d3 ", " d3 ", " d3 ", 24\n" \
  "v_add_u32 " c0 ", " c0 ", " d0 "\n v_add_u32 " c1 ", " c1 ", " d1 "\n v_add_u32 " c2 ", " c2 ", " d2 "\n v_add_u32 " c3 ", " c3 ", " d3 "\n" \
  "v_xor_b32 " b0 ", " b0 ", " c0 "\n v_xor_b32 " b1 ", " b1 ", " c1 "\n v_xor_b32 " b2 ", " b2 ", " c2 "\n v_xor_b32 " b3 ", " b3 ", " c3 "\n" \
  "v_alignbit_b32 " b0 ", " b0 ", " b0 ", 25\n v_alignbit_b32 " b1 ", " b1 ", " b1 ", 25\n v_alignbit_b32 " b2 ", " b2 ", " b2 ", 25\n v_alignbit_b32 " b3 ", " b3 ", " b3 ", 25\n"


// ROW map registers (bank = row r): x[4r+c] = v(40 + 4c + r)
#define R00 "v40"
#define R01 "v44"
#define R02 "v48"
#define R03 "v52"
#define R10 "v41"
#define R11 "v45"
#define R12 "v49"
#define R13 "v53"
#define R20 "v42"
#define R21 "v46"
#define R22 "v50"
#define R23 "v54"
#define R30 "v43"
#define R31 "v47"
#define R32 "v51"
#define R33 "v55"
// COL map registers (bank = column c): x[4r+c] = v(40 + 4r + c)
#define C00 "v40"
#define C01 "v41"
#define C02 "v42"
#define C03 "v43"
#define C10 "v44"
#define C11 "v45"
#define C12 "v46"
#define C13 "v47"
#define C20 "v48"
#define C21 "v49"
#define C22 "v50"
#define C23 "v51"
#define C30 "v52"
#define C31 "v53"
#define C32 "v54"
#define C33 "v55"

#define DR(M)                                                                                                       \
  QR4(M##00, M##10, M##20, M##30, M##01, M##11, M##21, M##31, M##02, M##12, M##22, M##32, M##03, M##13, M##23, M##33) \
  QR4(M##00, M##11, M##22, M##33, M##01, M##12, M##23, M##30, M##02, M##13, M##20, M##31, M##03, M##10, M##21, M##32)


// the same dependency pattern without the rotates (add/xor only) and rotates alone
#define QR4_NOROT(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3)                        \
  "v_add_u32 " a0 ", " a0 ", " b0 "\n v_add_u32 " a1 ", " a1 ", " b1 "\n v_add_u32 " a2 ", " a2 ", " b2 "\n v_add_u32 " a3 ", " a3 ", " b3 "\n" \
  "v_xor_b32 " d0 ", " d0 ", " a0 "\n v_xor_b32 " d1 ", " d1 ", " a1 "\n v_xor_b32 " d2 ", " d2 ", " a2 "\n v_xor_b32 " d3 ", " d3 ", " a3 "\n" \
  "v_add_u32 " c0 ", " c0 ", " d0 "\n v_add_u32 " c1 ", " c1 ", " d1 "\n v_add_u32 " c2 ", " c2 ", " d2 "\n v_add_u32 " c3 ", " c3 ", " d3 "\n" \
  "v_xor_b32 " b0 ", " b0 ", " c0 "\n v_xor_b32 " b1 ", " b1 ", " c1 "\n v_xor_b32 " b2 ", " b2 ", " c2 "\n v_xor_b32 " b3 ", " b3 ", " c3 "\n" \
  "v_add_u32 " a0 ", " a0 ", " b0 "\n v_add_u32 " a1 ", " a1 ", " b1 "\n v_add_u32 " a2 ", " a2 ", " b2 "\n v_add_u32 " a3 ", " a3 ", " b3 "\n" \
  "v_xor_b32 " d0 ", " d0 ", " a0 "\n v_xor_b32 " d1 ", " d1 ", " a1 "\n v_xor_b32 " d2 ", " d2 ", " a2 "\n v_xor_b32 " d3 ", " d3 ", " a3 "\n" \
  "v_add_u32 " c0 ", " c0 ", " d0 "\n v_add_u32 " c1 ", " c1 ", " d1 "\n v_add_u32 " c2 ", " c2 ", " d2 "\n v_add_u32 " c3 ", " c3 ", " d3 "\n" \
  "v_xor_b32 " b0 ", " b0 ", " c0 "\n v_xor_b32 " b1 ", " b1 ", " c1 "\n v_xor_b32 " b2 ", " b2 ", " c2 "\n v_xor_b32 " b3 ", " b3 ", " c3 "\n"
#define DR_NOROT(M)                                                                                                       \
  QR4_NOROT(M##00, M##10, M##20, M##30, M##01, M##11, M##21, M##31, M##02, M##12, M##22, M##32, M##03, M##13, M##23, M##33) \
  QR4_NOROT(M##00, M##11, M##22, M##33, M##01, M##12, M##23, M##30, M##02, M##13, M##20, M##31, M##03, M##10, M##21, M##32)
#define ROT16                                                                                             \
  "v_alignbit_b32 v40, v40, v40, 20\n v_alignbit_b32 v41, v41, v41, 20\n v_alignbit_b32 v42, v42, v42, 20\n v_alignbit_b32 v43, v43, v43, 20\n" \
  "v_alignbit_b32 v44, v44, v44, 20\n v_alignbit_b32 v45, v45, v45, 20\n v_alignbit_b32 v46, v46, v46, 20\n v_alignbit_b32 v47, v47, v47, 20\n" \
  "v_alignbit_b32 v48, v48, v48, 20\n v_alignbit_b32 v49, v49, v49, 20\n v_alignbit_b32 v50, v50, v50, 20\n v_alignbit_b32 v51, v51, v51, 20\n" \
  "v_alignbit_b32 v52, v52, v52, 20\n v_alignbit_b32 v53, v53, v53, 20\n v_alignbit_b32 v54, v54, v54, 20\n v_alignbit_b32 v55, v55, v55, 20\n"
// add and alignbit alternating, independent (no dependency between neighbours)
#define MIX16                                                                                             \
  "v_add_u32 v40, v40, v56\n v_alignbit_b32 v41, v41, v41, 20\n v_add_u32 v42, v42, v57\n v_alignbit_b32 v43, v43, v43, 20\n" \
  "v_add_u32 v44, v44, v58\n v_alignbit_b32 v45, v45, v45, 20\n v_add_u32 v46, v46, v59\n v_alignbit_b32 v47, v47, v47, 20\n" \
  "v_add_u32 v48, v48, v60\n v_alignbit_b32 v49, v49, v49, 20\n v_add_u32 v50, v50, v61\n v_alignbit_b32 v51, v51, v51, 20\n" \
  "v_add_u32 v52, v52, v62\n v_alignbit_b32 v53, v53, v53, 20\n v_add_u32 v54, v54, v63\n v_alignbit_b32 v55, v55, v55, 20\n"
// add, xor, xor (VOP2) then one alignbit: the ChaCha ratio, independent ops
#define MIX3_1                                                                                            \
  "v_add_u32 v40, v40, v56\n v_xor_b32 v41, v41, v57\n v_alignbit_b32 v42, v42, v42, 20\n" \
  "v_add_u32 v43, v43, v58\n v_xor_b32 v44, v44, v59\n v_alignbit_b32 v45, v45, v45, 20\n" \
  "v_add_u32 v46, v46, v60\n v_xor_b32 v47, v47, v61\n v_alignbit_b32 v48, v48, v48, 20\n" \
  "v_add_u32 v49, v49, v62\n v_xor_b32 v50, v50, v63\n v_alignbit_b32 v51, v51, v51, 20\n"


// ---- VOP2-only quarter-round variants (generated op lists) --------------------------------
// rotl(x, n) as three VOP2 ops through a temp; rotl16 of (d ^ a) as two SDWA xors
#define DR_SHIFT \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_e32 v43, v43, v40\n" \
  "v_xor_b32_e32 v47, v47, v44\n" \
  "v_xor_b32_e32 v51, v51, v48\n" \
  "v_xor_b32_e32 v55, v55, v52\n" \
  "v_lshlrev_b32_e32 v56, 16, v43\n" \
  "v_lshlrev_b32_e32 v57, 16, v47\n" \
  "v_lshlrev_b32_e32 v58, 16, v51\n" \
  "v_lshlrev_b32_e32 v59, 16, v55\n" \
  "v_lshrrev_b32_e32 v43, 16, v43\n" \
  "v_lshrrev_b32_e32 v47, 16, v47\n" \
  "v_lshrrev_b32_e32 v51, 16, v51\n" \
  "v_lshrrev_b32_e32 v55, 16, v55\n" \
  "v_or_b32_e32 v43, v43, v56\n" \
  "v_or_b32_e32 v47, v47, v57\n" \
  "v_or_b32_e32 v51, v51, v58\n" \
  "v_or_b32_e32 v55, v55, v59\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_lshlrev_b32_e32 v56, 12, v41\n" \
  "v_lshlrev_b32_e32 v57, 12, v45\n" \
  "v_lshlrev_b32_e32 v58, 12, v49\n" \
  "v_lshlrev_b32_e32 v59, 12, v53\n" \
  "v_lshrrev_b32_e32 v41, 20, v41\n" \
  "v_lshrrev_b32_e32 v45, 20, v45\n" \
  "v_lshrrev_b32_e32 v49, 20, v49\n" \
  "v_lshrrev_b32_e32 v53, 20, v53\n" \
  "v_or_b32_e32 v41, v41, v56\n" \
  "v_or_b32_e32 v45, v45, v57\n" \
  "v_or_b32_e32 v49, v49, v58\n" \
  "v_or_b32_e32 v53, v53, v59\n" \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_e32 v43, v43, v40\n" \
  "v_xor_b32_e32 v47, v47, v44\n" \
  "v_xor_b32_e32 v51, v51, v48\n" \
  "v_xor_b32_e32 v55, v55, v52\n" \
  "v_lshlrev_b32_e32 v56, 8, v43\n" \
  "v_lshlrev_b32_e32 v57, 8, v47\n" \
  "v_lshlrev_b32_e32 v58, 8, v51\n" \
  "v_lshlrev_b32_e32 v59, 8, v55\n" \
  "v_lshrrev_b32_e32 v43, 24, v43\n" \
  "v_lshrrev_b32_e32 v47, 24, v47\n" \
  "v_lshrrev_b32_e32 v51, 24, v51\n" \
  "v_lshrrev_b32_e32 v55, 24, v55\n" \
  "v_or_b32_e32 v43, v43, v56\n" \
  "v_or_b32_e32 v47, v47, v57\n" \
  "v_or_b32_e32 v51, v51, v58\n" \
  "v_or_b32_e32 v55, v55, v59\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_lshlrev_b32_e32 v56, 7, v41\n" \
  "v_lshlrev_b32_e32 v57, 7, v45\n" \
  "v_lshlrev_b32_e32 v58, 7, v49\n" \
  "v_lshlrev_b32_e32 v59, 7, v53\n" \
  "v_lshrrev_b32_e32 v41, 25, v41\n" \
  "v_lshrrev_b32_e32 v45, 25, v45\n" \
  "v_lshrrev_b32_e32 v49, 25, v49\n" \
  "v_lshrrev_b32_e32 v53, 25, v53\n" \
  "v_or_b32_e32 v41, v41, v56\n" \
  "v_or_b32_e32 v45, v45, v57\n" \
  "v_or_b32_e32 v49, v49, v58\n" \
  "v_or_b32_e32 v53, v53, v59\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_e32 v55, v55, v40\n" \
  "v_xor_b32_e32 v43, v43, v44\n" \
  "v_xor_b32_e32 v47, v47, v48\n" \
  "v_xor_b32_e32 v51, v51, v52\n" \
  "v_lshlrev_b32_e32 v56, 16, v55\n" \
  "v_lshlrev_b32_e32 v57, 16, v43\n" \
  "v_lshlrev_b32_e32 v58, 16, v47\n" \
  "v_lshlrev_b32_e32 v59, 16, v51\n" \
  "v_lshrrev_b32_e32 v55, 16, v55\n" \
  "v_lshrrev_b32_e32 v43, 16, v43\n" \
  "v_lshrrev_b32_e32 v47, 16, v47\n" \
  "v_lshrrev_b32_e32 v51, 16, v51\n" \
  "v_or_b32_e32 v55, v55, v56\n" \
  "v_or_b32_e32 v43, v43, v57\n" \
  "v_or_b32_e32 v47, v47, v58\n" \
  "v_or_b32_e32 v51, v51, v59\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_lshlrev_b32_e32 v56, 12, v45\n" \
  "v_lshlrev_b32_e32 v57, 12, v49\n" \
  "v_lshlrev_b32_e32 v58, 12, v53\n" \
  "v_lshlrev_b32_e32 v59, 12, v41\n" \
  "v_lshrrev_b32_e32 v45, 20, v45\n" \
  "v_lshrrev_b32_e32 v49, 20, v49\n" \
  "v_lshrrev_b32_e32 v53, 20, v53\n" \
  "v_lshrrev_b32_e32 v41, 20, v41\n" \
  "v_or_b32_e32 v45, v45, v56\n" \
  "v_or_b32_e32 v49, v49, v57\n" \
  "v_or_b32_e32 v53, v53, v58\n" \
  "v_or_b32_e32 v41, v41, v59\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_e32 v55, v55, v40\n" \
  "v_xor_b32_e32 v43, v43, v44\n" \
  "v_xor_b32_e32 v47, v47, v48\n" \
  "v_xor_b32_e32 v51, v51, v52\n" \
  "v_lshlrev_b32_e32 v56, 8, v55\n" \
  "v_lshlrev_b32_e32 v57, 8, v43\n" \
  "v_lshlrev_b32_e32 v58, 8, v47\n" \
  "v_lshlrev_b32_e32 v59, 8, v51\n" \
  "v_lshrrev_b32_e32 v55, 24, v55\n" \
  "v_lshrrev_b32_e32 v43, 24, v43\n" \
  "v_lshrrev_b32_e32 v47, 24, v47\n" \
  "v_lshrrev_b32_e32 v51, 24, v51\n" \
  "v_or_b32_e32 v55, v55, v56\n" \
  "v_or_b32_e32 v43, v43, v57\n" \
  "v_or_b32_e32 v47, v47, v58\n" \
  "v_or_b32_e32 v51, v51, v59\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_lshlrev_b32_e32 v56, 7, v45\n" \
  "v_lshlrev_b32_e32 v57, 7, v49\n" \
  "v_lshlrev_b32_e32 v58, 7, v53\n" \
  "v_lshlrev_b32_e32 v59, 7, v41\n" \
  "v_lshrrev_b32_e32 v45, 25, v45\n" \
  "v_lshrrev_b32_e32 v49, 25, v49\n" \
  "v_lshrrev_b32_e32 v53, 25, v53\n" \
  "v_lshrrev_b32_e32 v41, 25, v41\n" \
  "v_or_b32_e32 v45, v45, v56\n" \
  "v_or_b32_e32 v49, v49, v57\n" \
  "v_or_b32_e32 v53, v53, v58\n" \
  "v_or_b32_e32 v41, v41, v59\n"
constexpr int DR_SHIFT_n = 160;
#define DR_SDWA \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_sdwa v56, v43, v40 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v57, v47, v44 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v58, v51, v48 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v59, v55, v52 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v56, v43, v40 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v57, v47, v44 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v58, v51, v48 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v59, v55, v52 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_mov_b32_e32 v43, v56\n" \
  "v_mov_b32_e32 v47, v57\n" \
  "v_mov_b32_e32 v51, v58\n" \
  "v_mov_b32_e32 v55, v59\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_lshlrev_b32_e32 v56, 12, v41\n" \
  "v_lshlrev_b32_e32 v57, 12, v45\n" \
  "v_lshlrev_b32_e32 v58, 12, v49\n" \
  "v_lshlrev_b32_e32 v59, 12, v53\n" \
  "v_lshrrev_b32_e32 v41, 20, v41\n" \
  "v_lshrrev_b32_e32 v45, 20, v45\n" \
  "v_lshrrev_b32_e32 v49, 20, v49\n" \
  "v_lshrrev_b32_e32 v53, 20, v53\n" \
  "v_or_b32_e32 v41, v41, v56\n" \
  "v_or_b32_e32 v45, v45, v57\n" \
  "v_or_b32_e32 v49, v49, v58\n" \
  "v_or_b32_e32 v53, v53, v59\n" \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_e32 v43, v43, v40\n" \
  "v_xor_b32_e32 v47, v47, v44\n" \
  "v_xor_b32_e32 v51, v51, v48\n" \
  "v_xor_b32_e32 v55, v55, v52\n" \
  "v_lshlrev_b32_e32 v56, 8, v43\n" \
  "v_lshlrev_b32_e32 v57, 8, v47\n" \
  "v_lshlrev_b32_e32 v58, 8, v51\n" \
  "v_lshlrev_b32_e32 v59, 8, v55\n" \
  "v_lshrrev_b32_e32 v43, 24, v43\n" \
  "v_lshrrev_b32_e32 v47, 24, v47\n" \
  "v_lshrrev_b32_e32 v51, 24, v51\n" \
  "v_lshrrev_b32_e32 v55, 24, v55\n" \
  "v_or_b32_e32 v43, v43, v56\n" \
  "v_or_b32_e32 v47, v47, v57\n" \
  "v_or_b32_e32 v51, v51, v58\n" \
  "v_or_b32_e32 v55, v55, v59\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_lshlrev_b32_e32 v56, 7, v41\n" \
  "v_lshlrev_b32_e32 v57, 7, v45\n" \
  "v_lshlrev_b32_e32 v58, 7, v49\n" \
  "v_lshlrev_b32_e32 v59, 7, v53\n" \
  "v_lshrrev_b32_e32 v41, 25, v41\n" \
  "v_lshrrev_b32_e32 v45, 25, v45\n" \
  "v_lshrrev_b32_e32 v49, 25, v49\n" \
  "v_lshrrev_b32_e32 v53, 25, v53\n" \
  "v_or_b32_e32 v41, v41, v56\n" \
  "v_or_b32_e32 v45, v45, v57\n" \
  "v_or_b32_e32 v49, v49, v58\n" \
  "v_or_b32_e32 v53, v53, v59\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_sdwa v56, v55, v40 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v57, v43, v44 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v58, v47, v48 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v59, v51, v52 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_xor_b32_sdwa v56, v55, v40 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v57, v43, v44 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v58, v47, v48 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa v59, v51, v52 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_mov_b32_e32 v55, v56\n" \
  "v_mov_b32_e32 v43, v57\n" \
  "v_mov_b32_e32 v47, v58\n" \
  "v_mov_b32_e32 v51, v59\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_lshlrev_b32_e32 v56, 12, v45\n" \
  "v_lshlrev_b32_e32 v57, 12, v49\n" \
  "v_lshlrev_b32_e32 v58, 12, v53\n" \
  "v_lshlrev_b32_e32 v59, 12, v41\n" \
  "v_lshrrev_b32_e32 v45, 20, v45\n" \
  "v_lshrrev_b32_e32 v49, 20, v49\n" \
  "v_lshrrev_b32_e32 v53, 20, v53\n" \
  "v_lshrrev_b32_e32 v41, 20, v41\n" \
  "v_or_b32_e32 v45, v45, v56\n" \
  "v_or_b32_e32 v49, v49, v57\n" \
  "v_or_b32_e32 v53, v53, v58\n" \
  "v_or_b32_e32 v41, v41, v59\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_e32 v55, v55, v40\n" \
  "v_xor_b32_e32 v43, v43, v44\n" \
  "v_xor_b32_e32 v47, v47, v48\n" \
  "v_xor_b32_e32 v51, v51, v52\n" \
  "v_lshlrev_b32_e32 v56, 8, v55\n" \
  "v_lshlrev_b32_e32 v57, 8, v43\n" \
  "v_lshlrev_b32_e32 v58, 8, v47\n" \
  "v_lshlrev_b32_e32 v59, 8, v51\n" \
  "v_lshrrev_b32_e32 v55, 24, v55\n" \
  "v_lshrrev_b32_e32 v43, 24, v43\n" \
  "v_lshrrev_b32_e32 v47, 24, v47\n" \
  "v_lshrrev_b32_e32 v51, 24, v51\n" \
  "v_or_b32_e32 v55, v55, v56\n" \
  "v_or_b32_e32 v43, v43, v57\n" \
  "v_or_b32_e32 v47, v47, v58\n" \
  "v_or_b32_e32 v51, v51, v59\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_lshlrev_b32_e32 v56, 7, v45\n" \
  "v_lshlrev_b32_e32 v57, 7, v49\n" \
  "v_lshlrev_b32_e32 v58, 7, v53\n" \
  "v_lshlrev_b32_e32 v59, 7, v41\n" \
  "v_lshrrev_b32_e32 v45, 25, v45\n" \
  "v_lshrrev_b32_e32 v49, 25, v49\n" \
  "v_lshrrev_b32_e32 v53, 25, v53\n" \
  "v_lshrrev_b32_e32 v41, 25, v41\n" \
  "v_or_b32_e32 v45, v45, v56\n" \
  "v_or_b32_e32 v49, v49, v57\n" \
  "v_or_b32_e32 v53, v53, v58\n" \
  "v_or_b32_e32 v41, v41, v59\n"
constexpr int DR_SDWA_n = 152;
#define DR_ALIGN2 \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_e32 v43, v43, v40\n" \
  "v_xor_b32_e32 v47, v47, v44\n" \
  "v_xor_b32_e32 v51, v51, v48\n" \
  "v_xor_b32_e32 v55, v55, v52\n" \
  "v_alignbit_b32 v43, v43, v43, 16\n" \
  "v_alignbit_b32 v47, v47, v47, 16\n" \
  "v_alignbit_b32 v51, v51, v51, 16\n" \
  "v_alignbit_b32 v55, v55, v55, 16\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_alignbit_b32 v41, v41, v41, 20\n" \
  "v_alignbit_b32 v45, v45, v45, 20\n" \
  "v_alignbit_b32 v49, v49, v49, 20\n" \
  "v_alignbit_b32 v53, v53, v53, 20\n" \
  "v_add_u32_e32 v40, v40, v41\n" \
  "v_add_u32_e32 v44, v44, v45\n" \
  "v_add_u32_e32 v48, v48, v49\n" \
  "v_add_u32_e32 v52, v52, v53\n" \
  "v_xor_b32_e32 v43, v43, v40\n" \
  "v_xor_b32_e32 v47, v47, v44\n" \
  "v_xor_b32_e32 v51, v51, v48\n" \
  "v_xor_b32_e32 v55, v55, v52\n" \
  "v_alignbit_b32 v43, v43, v43, 24\n" \
  "v_alignbit_b32 v47, v47, v47, 24\n" \
  "v_alignbit_b32 v51, v51, v51, 24\n" \
  "v_alignbit_b32 v55, v55, v55, 24\n" \
  "v_add_u32_e32 v42, v42, v43\n" \
  "v_add_u32_e32 v46, v46, v47\n" \
  "v_add_u32_e32 v50, v50, v51\n" \
  "v_add_u32_e32 v54, v54, v55\n" \
  "v_xor_b32_e32 v41, v41, v42\n" \
  "v_xor_b32_e32 v45, v45, v46\n" \
  "v_xor_b32_e32 v49, v49, v50\n" \
  "v_xor_b32_e32 v53, v53, v54\n" \
  "v_alignbit_b32 v41, v41, v41, 25\n" \
  "v_alignbit_b32 v45, v45, v45, 25\n" \
  "v_alignbit_b32 v49, v49, v49, 25\n" \
  "v_alignbit_b32 v53, v53, v53, 25\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_e32 v55, v55, v40\n" \
  "v_xor_b32_e32 v43, v43, v44\n" \
  "v_xor_b32_e32 v47, v47, v48\n" \
  "v_xor_b32_e32 v51, v51, v52\n" \
  "v_alignbit_b32 v55, v55, v55, 16\n" \
  "v_alignbit_b32 v43, v43, v43, 16\n" \
  "v_alignbit_b32 v47, v47, v47, 16\n" \
  "v_alignbit_b32 v51, v51, v51, 16\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_alignbit_b32 v45, v45, v45, 20\n" \
  "v_alignbit_b32 v49, v49, v49, 20\n" \
  "v_alignbit_b32 v53, v53, v53, 20\n" \
  "v_alignbit_b32 v41, v41, v41, 20\n" \
  "v_add_u32_e32 v40, v40, v45\n" \
  "v_add_u32_e32 v44, v44, v49\n" \
  "v_add_u32_e32 v48, v48, v53\n" \
  "v_add_u32_e32 v52, v52, v41\n" \
  "v_xor_b32_e32 v55, v55, v40\n" \
  "v_xor_b32_e32 v43, v43, v44\n" \
  "v_xor_b32_e32 v47, v47, v48\n" \
  "v_xor_b32_e32 v51, v51, v52\n" \
  "v_alignbit_b32 v55, v55, v55, 24\n" \
  "v_alignbit_b32 v43, v43, v43, 24\n" \
  "v_alignbit_b32 v47, v47, v47, 24\n" \
  "v_alignbit_b32 v51, v51, v51, 24\n" \
  "v_add_u32_e32 v50, v50, v55\n" \
  "v_add_u32_e32 v54, v54, v43\n" \
  "v_add_u32_e32 v42, v42, v47\n" \
  "v_add_u32_e32 v46, v46, v51\n" \
  "v_xor_b32_e32 v45, v45, v50\n" \
  "v_xor_b32_e32 v49, v49, v54\n" \
  "v_xor_b32_e32 v53, v53, v42\n" \
  "v_xor_b32_e32 v41, v41, v46\n" \
  "v_alignbit_b32 v45, v45, v45, 25\n" \
  "v_alignbit_b32 v49, v49, v49, 25\n" \
  "v_alignbit_b32 v53, v53, v53, 25\n" \
  "v_alignbit_b32 v41, v41, v41, 25\n"
constexpr int DR_ALIGN2_n = 96;
#define CLOB                                                                                                     \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
      "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

#define KERNEL(name, body, ninst)                                                                  \
  __global__ void __launch_bounds__(256) name(uint32_t iters, uint32_t* out, uint64_t* clk) {        \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                                    \
    for (uint32_t i = 0; i < iters; ++i) {                                                         \
      asm volatile(body ::: CLOB);                                                                 \
    }                                                                                              \
    uint32_t r;                                                                                    \
    asm volatile("v_mov_b32 %0, v40" : "=v"(r)::CLOB);                                             \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                                    \
    if (r == 0x12345678u) out[threadIdx.x] = r;                                                    \
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;                                     \
  }                                                                                                \
  constexpr int name##_n = ninst;

KERNEL(k_add_same, ADD_SAME ADD_SAME ADD_SAME ADD_SAME, 64)
KERNEL(k_add_diff, ADD_DIFF ADD_DIFF ADD_DIFF ADD_DIFF, 64)
KERNEL(k_qr_row, DR(R) DR(R), 192)
KERNEL(k_qr_col, DR(C) DR(C), 192)
KERNEL(k_qr_norot, DR_NOROT(R) DR_NOROT(R), 128)
KERNEL(k_rot, ROT16 ROT16 ROT16 ROT16, 64)
KERNEL(k_mix16, MIX16 MIX16 MIX16 MIX16, 64)
KERNEL(k_mix3, MIX3_1 MIX3_1 MIX3_1 MIX3_1, 48)
KERNEL(k_dr_shift, DR_SHIFT DR_SHIFT, 2 * DR_SHIFT_n)
KERNEL(k_dr_sdwa, DR_SDWA DR_SDWA, 2 * DR_SDWA_n)
KERNEL(k_dr_align, DR_ALIGN2 DR_ALIGN2, 2 * DR_ALIGN2_n)

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  uint64_t* clk;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&clk, 64);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t iters = 4000;
  const int blocks = cus * 8;  // 8 waves per SIMD (4 waves per block, 8 blocks per CU)
  auto run = [&](const char* nm, void (*k)(uint32_t, uint32_t*, uint64_t*), int n) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, iters, out, clk);
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, iters, out, clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t c = 0;
    (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    const double wave_inst_per_simd = (double)iters * n * 8.0;  // 8 waves per SIMD
    const double cyc = (double)c;                                // shader cycles of one wave's loop
    printf("%-10s %5d inst %8.3f ms/launch  %6.3f cycles per wave-instruction per SIMD (s_memtime)  %6.3f at 2.4 GHz\n", nm, n,
           ms / reps, cyc / wave_inst_per_simd, ms / reps * 1e-3 * 2.4e9 / wave_inst_per_simd);
  };
  run("add_same", k_add_same, k_add_same_n);
  run("add_diff", k_add_diff, k_add_diff_n);
  run("qr_row", k_qr_row, k_qr_row_n);
  run("qr_col", k_qr_col, k_qr_col_n);
  run("qr_norot", k_qr_norot, k_qr_norot_n);
  run("rot", k_rot, k_rot_n);
  run("add|rot", k_mix16, k_mix16_n);
  run("add,xor,rot", k_mix3, k_mix3_n);
  // per double round (96 ChaCha ops): time per DR = n * cycles
  run("dr_shift", k_dr_shift, k_dr_shift_n);
  run("dr_sdwa", k_dr_sdwa, k_dr_sdwa_n);
  run("dr_align", k_dr_align, k_dr_align_n);
  return 0;
}
