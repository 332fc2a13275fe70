// hrl_split.h — exact three-way bf16 split of fp32 MFMA operands (gfx950), shared by the board and torus convs.
//
// x = h + m + l EXACTLY: h = x with the low 16 bits cleared (8 significant bits), r = x - h is exact
// (<= 16 significant bits), m = r with the low 16 bits cleared, l = r - m is exact and has <= 8
// significant bits, so it is a bf16 as is.  A product x*w keeps the six terms hh, hm, mh, hl, lh, mm;
// the dropped ml, lm, ll are below 2^-23 |x w| together -- the size of one fp32 rounding.  Every
// bf16 x bf16 product is exact in fp32 and the MFMA accumulates in fp32, so the result is
// fp32-accurate, at 6/16 of the fp32 MFMA's cycles (gfx950: v_mfma_f32_16x16x4_f32 runs at 1/16 of
// the bf16 rate, MI355X_MICROARCH.md; v_mfma_f32_16x16x32_bf16 takes 16 cycles, tools/micro/mfma_rate.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hrl_split {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float x, uint32_t &h, uint32_t &m, uint32_t &l) {
    const uint32_t hb = __float_as_uint(x) & 0xffff0000u;
    const float r = x - __uint_as_float(hb);
    const uint32_t mb = __float_as_uint(r) & 0xffff0000u;
    h = hb >> 16;
    m = mb >> 16;
    l = __float_as_uint(r - __uint_as_float(mb)) >> 16;
}

// the exact split of two values (rows 2k and 2k+1 of an MFMA operand) packed as bf16 pairs: H = {h0, h1},
// M = {m0, m1}, L = {l0, l1} (x0 in the low half).  The same parts as split3, in 11 VALU instead of 20: the parts
// are kept as fp32 bit patterns whose low 16 bits are zero, and v_perm_b32 takes both high halves at once.
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t &H, uint32_t &M, uint32_t &L) {
    const uint32_t hb0 = __float_as_uint(x0) & 0xffff0000u, hb1 = __float_as_uint(x1) & 0xffff0000u;
    const float r0 = x0 - __uint_as_float(hb0), r1 = x1 - __uint_as_float(hb1);
    const uint32_t mb0 = __float_as_uint(r0) & 0xffff0000u, mb1 = __float_as_uint(r1) & 0xffff0000u;
    const uint32_t lb0 = __float_as_uint(r0 - __uint_as_float(mb0));
    const uint32_t lb1 = __float_as_uint(r1 - __uint_as_float(mb1));
    // perm(S0, S1, sel): selector bytes 0-3 pick S1's bytes, 4-7 S0's: {S1.b2, S1.b3, S0.b2, S0.b3}
    H = __builtin_amdgcn_perm(hb1, hb0, 0x07060302u);
    M = __builtin_amdgcn_perm(mb1, mb0, 0x07060302u);
    L = __builtin_amdgcn_perm(lb1, lb0, 0x07060302u);
}

// part 0/1/2 (h/m/l) of x as the 16 bf16 bits
__device__ __forceinline__ uint32_t split_part(float x, int part) {
    uint32_t h, m, l;
    split3(x, h, m, l);
    return part == 0 ? h : (part == 1 ? m : l);
}

// 8 fp32 (one lane's k-run of a 16x16x32 operand) -> the h/m/l bf16x8 fragments
__device__ __forceinline__ void split8(const float (&v)[8], uint4 &H, uint4 &M, uint4 &L) {
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split3(v[2 * d], h0, m0, l0);
        split3(v[2 * d + 1], h1, m1, l1);
        h[d] = h0 | (h1 << 16);
        m[d] = m0 | (m1 << 16);
        l[d] = l0 | (l1 << 16);
    }
    H = make_uint4(h[0], h[1], h[2], h[3]);
    M = make_uint4(m[0], m[1], m[2], m[3]);
    L = make_uint4(l[0], l[1], l[2], l[3]);
}

__device__ __forceinline__ f32x4 mfma_bf16(const uint4 &a, const uint4 &b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                   c, 0, 0, 0);
}

// c += A * B with both operands as exact splits (smallest terms first)
__device__ __forceinline__ f32x4 mfma_split(const uint4 &Ah, const uint4 &Am, const uint4 &Al, const uint4 &Bh,
                                            const uint4 &Bm, const uint4 &Bl, f32x4 c) {
    c = mfma_bf16(Al, Bh, c);
    c = mfma_bf16(Am, Bm, c);
    c = mfma_bf16(Ah, Bl, c);
    c = mfma_bf16(Am, Bh, c);
    c = mfma_bf16(Ah, Bm, c);
    return mfma_bf16(Ah, Bh, c);
}

}  // namespace hrl_split
