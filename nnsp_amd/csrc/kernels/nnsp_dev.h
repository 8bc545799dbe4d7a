// nnsp_dev.h -- gfx950 device building blocks of the ns-nnsp hot path.
//
// Every function here reproduces the integer semantics of the reference C
// (ARM_OPTIMIZED=1 build, reference/ns-nnsp/src) or of CMSIS-DSP 1.10.0's
// arm_rfft_q31 bit for bit; file:line citations name the code each follows.
// Signed overflow wraps (as on the Cortex-M4): all such arithmetic goes
// through uint32 helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../gen/nnsp_tables.h"

namespace nnsp {

// ---- wrapping int32 helpers -------------------------------------------------
__device__ __forceinline__ int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
__device__ __forceinline__ int32_t wshl(int32_t a, int s) { return (int32_t)((uint32_t)a << s); }
__device__ __forceinline__ int32_t sat32(int64_t v) {
    return v > INT32_MAX ? INT32_MAX : (v < INT32_MIN ? INT32_MIN : (int32_t)v);
}
__device__ __forceinline__ int16_t sat16(int64_t v) {
    return v > 32767 ? (int16_t)32767 : (v < -32768 ? (int16_t)-32768 : (int16_t)v);
}
// (int32)(((int64)a*b) >> 32): v_mul_hi_i32
__device__ __forceinline__ int32_t mulhi(int32_t a, int32_t b) { return __mulhi(a, b); }

// acc + (int64)a*b as one v_mad_i64_i32 (the compiler otherwise hoists the
// sign extensions of loop-invariant operands and emits a 64x64 multiply)
__device__ __forceinline__ int64_t mad_i64_i32(int32_t a, int32_t b, int64_t acc) {
    int64_t r;
    uint64_t carry;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(acc));
    return r;
}

// sat32(x >> 15) for any int64 x: the shifted low word from one funnel shift,
// and the range check on the high word in 32-bit compares (x >> 15 fits int32
// iff x >> 46 = hi >> 14 is 0 or -1) -- no 64-bit compares (v_cmp_*_i64 issue
// at ~5x an add, profiles/microbench/valu_rates2)
__device__ __forceinline__ int32_t sat32_shr15(int64_t x) {
    const int32_t hi = (int32_t)(x >> 32);
    const int32_t y = (int32_t)__builtin_amdgcn_alignbit((uint32_t)hi, (uint32_t)x, 15);
    return (uint32_t)((hi >> 14) + 1) < 2u ? y : ((hi >> 31) ^ INT32_MAX);
}

// sat32(((int64)a * b + (int64)c * d) >> 15) for int16 a, b, c and int32 d
// (lstm.c's cell update): one v_mad_i64_i32 and sat32_shr15
__device__ __forceinline__ int32_t cell_q15(int32_t a, int32_t b, int32_t c, int32_t d) {
    return sat32_shr15(mad_i64_i32(c, d, (int64_t)(a * b)));
}

// The same for the LSTM's own gate ranges: i, f in [0, 32767] (sigmoid_fix
// outputs) and g in [-32767, 32767] (tanh_fix) with ANY int32 c.  Then
// |f*c + i*g| <= 32767 * 2^31 + 32767^2, and >> 15 stays within
// [-2147450879, 2147450878]: lstm.c's saturation never binds (f < 1 in Q15
// shrinks any c), so the cell is one v_mad_i64_i32 and one funnel shift
// (tests/test_cell_q15.py checks the bound and the equality)
__device__ __forceinline__ int32_t cell_q15_gates(int32_t i, int32_t g, int32_t f, int32_t c) {
    const int64_t x = mad_i64_i32(f, c, (int64_t)(i * g));
    return (int32_t)__builtin_amdgcn_alignbit((uint32_t)(x >> 32), (uint32_t)x, 15);
}

// SMMLAR / SMMULR contribution: floor((x*c + 2^31) / 2^32)
__device__ __forceinline__ int32_t rnd_add(int32_t x, int32_t c) {
    return (int32_t)(((int64_t)x * c + 0x80000000LL) >> 32);
}
// SMMLSR contribution: floor((2^31 - x*c) / 2^32) = -floor((x*c + 2^31 - 1) / 2^32)
__device__ __forceinline__ int32_t rnd_sub(int32_t x, int32_t c) {
    return (int32_t)(-(((int64_t)x * c + 0x7FFFFFFFLL) >> 32));
}

__device__ __forceinline__ int rev8(int i) { return (int)(__brev((uint32_t)i) >> 24); }

// Keep intra-wave LDS producer/consumer order (all lanes of one wave).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- radix-4 butterflies of arm_radix4_butterfly_q31 (CMSIS-DSP 1.10.0) -----
// first stage: inputs pre-scaled >>4, rotated outputs (..)<<1
// middle stages: sums >>2, rotated outputs (..)>>1 ; twiddles (co,si) k,2k,3k
struct Tw3 { int32_t c1, s1, c2, s2, c3, s3; };

__device__ __forceinline__ Tw3 load_tw3(int k) {
    Tw3 t;
    t.c1 = nnsp_tbl_tw256[2 * k];     t.s1 = nnsp_tbl_tw256[2 * k + 1];
    t.c2 = nnsp_tbl_tw256[4 * k];     t.s2 = nnsp_tbl_tw256[4 * k + 1];
    t.c3 = nnsp_tbl_tw256[6 * k];     t.s3 = nnsp_tbl_tw256[6 * k + 1];
    return t;
}

template <bool FIRST>
__device__ __forceinline__ void bfly4(int32_t& xa, int32_t& ya, int32_t& xb, int32_t& yb,
                                      int32_t& xc, int32_t& yc, int32_t& xd, int32_t& yd,
                                      const Tw3& w) {
    if (FIRST) {
        xa >>= 4; ya >>= 4; xb >>= 4; yb >>= 4; xc >>= 4; yc >>= 4; xd >>= 4; yd >>= 4;
    }
    int32_t r1 = wadd(xa, xc), r2 = wsub(xa, xc), s1 = wadd(ya, yc), s2 = wsub(ya, yc);
    int32_t t1 = wadd(xb, xd), t2 = wadd(yb, yd);
    const int32_t oa = FIRST ? wadd(r1, t1) : (wadd(r1, t1) >> 2);
    const int32_t pa = FIRST ? wadd(s1, t2) : (wadd(s1, t2) >> 2);
    r1 = wsub(r1, t1);
    s1 = wsub(s1, t2);
    t1 = wsub(yb, yd);
    t2 = wsub(xb, xd);
    int32_t ob = wadd(mulhi(r1, w.c2), mulhi(s1, w.s2));   // -> slot i1 ("xc'")
    int32_t pb = wsub(mulhi(s1, w.c2), mulhi(r1, w.s2));
    const int32_t q1 = wadd(r2, t1), q2 = wsub(r2, t1), u1 = wsub(s2, t2), u2 = wadd(s2, t2);
    int32_t oc = wadd(mulhi(q1, w.c1), mulhi(u1, w.s1));   // -> slot i2 ("xb'")
    int32_t pc = wsub(mulhi(u1, w.c1), mulhi(q1, w.s1));
    int32_t od = wadd(mulhi(q2, w.c3), mulhi(u2, w.s3));   // -> slot i3
    int32_t pd = wsub(mulhi(u2, w.c3), mulhi(q2, w.s3));
    if (FIRST) {
        ob = wshl(ob, 1); pb = wshl(pb, 1); oc = wshl(oc, 1); pc = wshl(pc, 1);
        od = wshl(od, 1); pd = wshl(pd, 1);
    } else {
        ob >>= 1; pb >>= 1; oc >>= 1; pc >>= 1; od >>= 1; pd >>= 1;
    }
    xa = oa; ya = pa; xb = ob; yb = pb; xc = oc; yc = pc; xd = od; yd = pd;
}

// last radix-4 stage: unscaled, outputs in slot order a, c', b', d'
__device__ __forceinline__ void bfly4_last(int32_t* q) {
    const int32_t xa = q[0], ya = q[1], xb = q[2], yb = q[3];
    const int32_t xc = q[4], yc = q[5], xd = q[6], yd = q[7];
    q[0] = wadd(wadd(xa, xb), wadd(xc, xd));
    q[1] = wadd(wadd(ya, yb), wadd(yc, yd));
    q[2] = wsub(wadd(xa, xc), wadd(xb, xd));
    q[3] = wsub(wadd(ya, yc), wadd(yb, yd));
    q[4] = wsub(wadd(xa, yb), wadd(xc, yd));
    q[5] = wsub(wadd(ya, xd), wadd(xb, yc));
    q[6] = wsub(wadd(xa, yd), wadd(yb, xc));
    q[7] = wsub(wadd(ya, xb), wadd(yc, xd));
}

// arm_split_rfft_q31 for one bin k in 1..255 (modifier 16):
// Z = bit-reversed cfft output; (xr,xi) = Z[k], (yr,yi) = Z[256-k]
__device__ __forceinline__ void split_bin(int32_t xr, int32_t xi, int32_t yr, int32_t yi,
                                          int32_t A1, int32_t A2, int32_t B1, int32_t& re,
                                          int32_t& im) {
    re = wadd(wadd(rnd_add(xr, A1), rnd_sub(xi, A2)), wadd(rnd_sub(yi, A2), rnd_add(yr, B1)));
    im = wadd(wadd(rnd_add(xr, A2), rnd_add(xi, A1)), wadd(rnd_sub(yi, B1), rnd_sub(yr, A2)));
}

// Bins k and 256-k together (k in 1..128).  CMSIS's coefficients are
// symmetric -- A1[256-k] = A1[k], A2[256-k] = -A2[k], B1[256-k] = B1[k] (checked
// by tests/test_tables.py) -- and rnd_sub(x, -c) = rnd_add(x, c), so bin 256-k
// is split_bin with x and y swapped and two of its eight rounded products,
// xr*A2 (SMMLAR) and yr*A2 (SMMLSR), are bin k's own: 14 products per pair.
//
// Each rounded product is one v_mad_i64_i32 with its rounding constant in an
// SGPR pair, its high word taken as is (rp_add: floor((x c + 2^31) / 2^32);
// rp_sub: floor((x c + 2^31 - 1) / 2^32), subtracted); the terms are then
// summed in 32 bits (v_add3 / v_sub).  Written as plain C the compiler chained
// each product's addend with the previous term's high word -- a v_mov and a
// 64-bit add per product, 18 extra VALU per frame.
__device__ __forceinline__ int32_t rp_hi(int32_t x, int32_t c, uint64_t k) {
    int64_t r;
    uint64_t carry;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(x), "v"(c), "s"(k));
    int32_t h = (int32_t)((uint64_t)r >> 32);
    asm("" : "+v"(h));   // an opaque high word: no re-association into 64-bit adds
    return h;
}
__device__ __forceinline__ int32_t rp_add(int32_t x, int32_t c) { return rp_hi(x, c, 0x80000000ull); }   // = rnd_add
__device__ __forceinline__ int32_t rp_sub(int32_t x, int32_t c) { return rp_hi(x, c, 0x7FFFFFFFull); }   // = -rnd_sub
__device__ __forceinline__ void split_pair(int32_t xr, int32_t xi, int32_t yr, int32_t yi, int32_t A1, int32_t A2,
                                           int32_t B1, int32_t& re0, int32_t& im0, int32_t& re1, int32_t& im1) {
    const int32_t xa2 = rp_add(xr, A2), ya2 = rp_sub(yr, A2);   // bin k's xr A2 (+), yr A2 (-)
    re0 = wsub(wadd(rp_add(xr, A1), rp_add(yr, B1)), wadd(rp_sub(xi, A2), rp_sub(yi, A2)));
    im0 = wsub(wadd(xa2, rp_add(xi, A1)), wadd(rp_sub(yi, B1), ya2));
    re1 = wadd(wadd(rp_add(yr, A1), rp_add(yi, A2)), wadd(rp_add(xi, A2), rp_add(xr, B1)));
    im1 = wsub(wadd(rp_add(yi, A1), xa2), wadd(ya2, rp_sub(xi, B1)));
}

// spec2pspec_arm (spectrogram_module.c:79-92): truncating cast of (re^2+im^2)>>27
__device__ __forceinline__ int32_t pspec_of(int32_t re, int32_t im) {
    return (int32_t)(((int64_t)re * re + (int64_t)im * im) >> 27);
}

// ---- the ARM_OPTIMIZED=0 build's FFT (row N4): fft.c:27-221, complex.c -----
// No saturation is reproduced: for int16 PCM the Frac15 window output is
// |x| <= 32767, so every FFT value stays below 256 * 2^15.5 < 2^24 and the
// split below 2^25 -- complex.c's int32 clamps (complex.c:29-31, 66-69) and
// rfft's (fft.c:108-111) never bind, and its 64-bit 4-point sums equal the
// wrapping int32 sums.
// complex32_complex16_elmtprod (complex.c:54-72): (z * w) >> 15, w a COMPLEX16
// word (real low, imag high); the low 32 bits of the shifted 64-bit sums
__device__ __forceinline__ void cmul15(int32_t& re, int32_t& im, uint32_t w) {
    const int32_t wr = (int32_t)(int16_t)(w & 0xffffu), wi = (int32_t)w >> 16;
    const int64_t R = mad_i64_i32(re, wr, mad_i64_i32(im, -wi, 0));
    const int64_t I = mad_i64_i32(re, wi, mad_i64_i32(im, wr, 0));
    re = (int32_t)((uint64_t)R >> 15);
    im = (int32_t)((uint64_t)I >> 15);
}

// one radix-4 DIF butterfly of fft() (fft.c:128-221): complex32_affine with
// M4 (fft.c:12-15) on (x0, x2, x1, x3), then every output -- r = 0 too -- times
// its twiddle tw[4k + r]; output r goes to slot idx + r N/4 (the same slots as
// bfly4: a, c', b', d')
__device__ __forceinline__ void bfly4_port(int32_t (&v)[8], uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    const int32_t xa = v[0], ya = v[1], xb = v[2], yb = v[3], xc = v[4], yc = v[5], xd = v[6], yd = v[7];
    const int32_t r1 = wadd(xa, xc), s1 = wadd(ya, yc), r2 = wsub(xa, xc), s2 = wsub(ya, yc);
    const int32_t t1 = wadd(xb, xd), u1 = wadd(yb, yd), t2 = wsub(yb, yd), u2 = wsub(xb, xd);
    v[0] = wadd(r1, t1); v[1] = wadd(s1, u1);   // x0 + x1 + x2 + x3
    v[2] = wsub(r1, t1); v[3] = wsub(s1, u1);   // x0 + x2 - x1 - x3
    v[4] = wadd(r2, t2); v[5] = wsub(s2, u2);   // x0 - x2 - j x1 + j x3
    v[6] = wsub(r2, t2); v[7] = wadd(s2, u2);   // x0 - x2 + j x1 - j x3
    cmul15(v[0], v[1], w0);
    cmul15(v[2], v[3], w1);
    cmul15(v[4], v[5], w2);
    cmul15(v[6], v[7], w3);
}

// rfft's split (fft.c:59-120) for bin i in 0..255: Z = the bit-reversed
// fft() output, (zr, zi) = Z[i], (nr, ni) = Z[(256 - i) & 255], w = rfft_tw[i]
__device__ __forceinline__ void split_bin_port(int32_t zr, int32_t zi, int32_t nr, int32_t ni, uint32_t w,
                                               int32_t& re, int32_t& im) {
    const int32_t tim = wsub(0, ni);
    const int32_t er = wadd(zr, nr) >> 1, ei = wadd(zi, tim) >> 1;
    int32_t orr = wsub(zi, tim) >> 1, oi = wsub(0, wsub(zr, nr)) >> 1;
    cmul15(orr, oi, w);
    re = wadd(orr, er);
    im = wadd(oi, ei);
}

// spec2pspec (spectrogram_module.c:33-45): truncating cast of (re^2+im^2)>>15
__device__ __forceinline__ int32_t pspec15_of(int32_t re, int32_t im) {
    return (int32_t)((uint64_t)mad_i64_i32(re, re, mad_i64_i32(im, im, 0)) >> 15);
}

// my_log10 + norm_oneTwo (fixlog10.c:9-50), bit_frac_in = 15
__device__ __forceinline__ int32_t log10_q15(int32_t x) {
    if (x == 0) x = 1;
    const uint32_t m = (uint32_t)x & 0x7FFFFFFFu;   // bits 30..0 searched
    int sh = 0;
    if (m) {
        const int b = 31 - __clz((int)m);
        sh = 15 - b;
    }
    const int32_t y = sh >= 0 ? wshl(x, sh) : (x >> -sh);
    const int e = -sh;
    int32_t kx = (y - 32768) >> 8;
    const int32_t dx = (y - 32768) - (kx << 8);
    kx = kx < 0 ? 0 : (kx > 127 ? 127 : kx);   // only x<0 (T3 wrap) leaves 0..127
    int32_t v = nnsp_tbl_log[2 * kx] + ((nnsp_tbl_log[2 * kx + 1] * dx) >> 15);
    v = (int32_t)(((int64_t)v * 0x3796) >> 15);
    return wadd(v, 0x2688 * e);
}

// ---- activations (activation.c) --------------------------------------------
__device__ __forceinline__ int16_t tanh_q15(int32_t x, const int16_t* tbl) {   // :31-69
    // branch-free form: the segment index is always in range (only |x| =
    // INT32_MIN, unreachable here, would index out of the reference's table)
    // and the (value, slope) pair is one 32-bit load
    const bool neg = x < 0;
    const int32_t a = neg ? wsub(0, x) : x;
    int32_t kx = wsub(a, 512) >> 10;
    kx = kx < 0 ? 0 : (kx > 191 ? 191 : kx);
    const int32_t dx = wsub(wsub(a, 512), kx << 10);
    const uint32_t pr = reinterpret_cast<const uint32_t*>(tbl)[kx];
    // dx is in [-512, 1023] whenever the result is used (|x| < 5*2^15 below),
    // so the 24-bit multiply (full rate) gives the exact 32-bit product
    const int32_t v = (int32_t)(int16_t)(pr & 0xffff) + (__mul24(dx, (int32_t)(int16_t)(pr >> 16)) >> 15);
    const int16_t y = a >= (5 << 15) ? (int16_t)0x7fff : (int16_t)(v > 0 ? v : 0);
    return neg ? (int16_t)-y : y;
}
__device__ __forceinline__ int16_t sigmoid_q15(int32_t x, const int16_t* tbl) {   // :72-87
    return (int16_t)((tanh_q15(x >> 1, tbl) >> 1) + 16384);
}
// tanh_q15 / sigmoid_q15 on the re-indexed table nnsp_tbl_tanh1 (tables.py
// tanh_interp_shifted; 256 (value, slope) pairs, the split NN kernels' LDS
// copy): the segment index (|x| + 512) >> 10 needs no clamp from below, the
// offset in the segment is (|x| + 512) & 1023, and the sign is restored with
// an xor and a subtract -- 15 VALU instead of ~19 (the LSTM gates evaluate
// five of these per unit and step).  Equal to tanh_q15 for every int32 but
// INT32_MIN (tests/test_tables.py, exhaustively over |x| < 2^18 and beyond).
__device__ __forceinline__ int32_t tanh_q15s_mag(int32_t a, const int16_t* tbl1) {   // a = |x| >= 0
    const uint32_t bb = (uint32_t)a + 512u;
    // (one v_bfe_u32 the compiler keeps: from the builtin it emits a shift,
    // a mask and an add for the scaled table offset instead of bfe + lshl_add)
    uint32_t kx;
    asm("v_bfe_u32 %0, %1, 10, 8" : "=v"(kx) : "v"(bb));
    const int32_t dx = (int32_t)(bb & 1023u);
    const uint32_t pr = reinterpret_cast<const uint32_t*>(tbl1)[kx];
    int32_t v = (int32_t)(int16_t)(pr & 0xffff) + (__mul24(dx, (int32_t)(int16_t)(pr >> 16)) >> 15);
    v = v > 0 ? v : 0;
    return a >= (5 << 15) ? 0x7fff : v;
}
__device__ __forceinline__ int16_t tanh_q15s(int32_t x, const int16_t* tbl1) {
    const int32_t s = x >> 31;
    const int32_t y = tanh_q15s_mag((x ^ s) - s, tbl1);
    return (int16_t)((y ^ s) - s);
}
__device__ __forceinline__ int16_t sigmoid_q15s(int32_t x, const int16_t* tbl1) {
    return (int16_t)((tanh_q15s(x >> 1, tbl1) >> 1) + 16384);
}
// tanh_fix / sigmoid_fix (activation.c:31-83) as one v_mad_i32_i24 on the
// affine table of tables.act_affine_table (nnsp_tbl_act), staged in LDS at tb:
// per half-segment j = bb >> 9 of bb = min(|x| + 512, 164352), 16 bytes
// (A_pos, b_pos, A_neg, b_neg); z = A + (bb & 511) * b is the reference's
// interpolation numerator with the sign, activation.c's max(., 0) and its
// saturation at 5 * 2^15 folded in.  F 0: tanh = z >> 15; F 1: sigmoid of the
// pre-shifted input w (sigmoid_fix(v) with w = v >> 1) = (z + 2^30) >>> 16.
// 12 / 13 VALU against 16 / 18 for tanh_q15s / sigmoid_q15s (one 5 KB table:
// a second, sigmoid-ready one would take S2I's recurrence past 160 KB of LDS);
// checked exhaustively in tests/test_tables.py
#define ACT_ENTRIES 322
#define ACT_BYTES (ACT_ENTRIES * 16)
template <int F>
__device__ __forceinline__ int32_t act_q15(int32_t x, const uint8_t* tb) {
    const uint32_t sgn = (uint32_t)x >> 31;
    const uint32_t xs = (uint32_t)(x ^ (x >> 31));   // |x| - sgn
    uint32_t bb = xs + 512u + sgn;
    bb = bb < 164352u ? bb : 164352u;
    const uint32_t off = ((bb >> 5) & 0x1ff0u) | (sgn << 3);
    const int2 e = *reinterpret_cast<const int2*>(tb + off);
    const int32_t z = __mul24((int32_t)(bb & 511u), e.y) + e.x;
    return F == 0 ? (z >> 15) : (int32_t)(((uint32_t)z + (1u << 30)) >> 16);
}
__device__ __forceinline__ int16_t relu6_q12(int32_t x) {   // :6-17
    int32_t v = x >> 3;
    v = v > 24576 ? 24576 : v;
    return (int16_t)(v < 0 ? 0 : v);
}

// development probes (NNSP_RECUR_CLOCKS): where a wave runs, packed as
// xcc << 12 | se << 8 | sh << 7 | cu << 3 | simd (HW_REG_HW_ID, HW_REG_XCC_ID)
__device__ __forceinline__ long long nnsp_hw_where() {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    return (long long)(((xcc & 15) << 12) | (se << 8) | (sh << 7) | (cu << 3) | simd);
}

enum { ACT_RELU6 = 0, ACT_TANH = 1, ACT_SIGMOID = 2, ACT_LINEAR = 3 };

// shift_64b / shift_32b (affine.c:565-591, affine_acc32b.c:566-592)
__device__ __forceinline__ int64_t shift64(int64_t v, int sh) {
    if (sh < 0) return v >> -sh;
    if (sh > 0) {
        const int64_t M = (int64_t)((1ULL << (63 - sh)) - 1), mn = -M - 1;
        v = v > M ? M : (v < mn ? mn : v);
        return (int64_t)((uint64_t)v << sh);
    }
    return v;
}
__device__ __forceinline__ int32_t shift32(int32_t v, int sh) {
    if (sh < 0) return v >> -sh;
    if (sh > 0) {
        const int32_t M = (int32_t)((1u << (31 - sh)) - 1), mn = -M - 1;
        v = v > M ? M : (v < mn ? mn : v);
        return wshl(v, sh);
    }
    return v;
}

// post-processing helpers (nn_speech.c:229-258)
__device__ __forceinline__ int32_t ceiling_q15(int32_t x) {
    const int32_t o = wshl(x >> 15, 15);
    return o == x ? o : wadd(o, 32768);
}
__device__ __forceinline__ int32_t pwr2_q15(int32_t x) {
    const int32_t c = ceiling_q15(x);
    const int32_t f = wsub(x, c);
    const int32_t sh = c >> 15;
    if (sh <= -15) return 0;
    const int32_t t = wadd(wshl(f, 1), 32768);
    int32_t o = 0x1fd7 + ((t * 0x057a) >> 15);
    o = 0x5a82 + ((t * o) >> 15);
    return sh < 0 ? (o >> -sh) : wshl(o, sh);
}

}  // namespace nnsp
