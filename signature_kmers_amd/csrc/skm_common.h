// skm_common.h -- shared host/device definitions for libskm (MI355X / gfx950).
//
// Key coding.  A build window is valid iff all 8 residues are in ok_prot_ (signature_build.h:102-103:
// the 20 amino acids in either case = 40 symbols).  Each symbol gets a code 0..39, and the window's
// code is the base-40 number k = sum c_j * 40^(7-j) < 40^8 < 2^43.  A bijective 43-bit mixer H
// spreads codes over buckets: the top bits of H(k) select owner GPU and level-1 bucket; the rest
// (`rem`) travels in the 8-byte occurrence record beside the packed-buffer position.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SKM_HD __host__ __device__ __forceinline__
#else
#define SKM_HD inline
#endif

namespace skm {

constexpr int K = 8;
constexpr int KEY_BITS = 43;
constexpr uint64_t KEY_MASK = (1ull << KEY_BITS) - 1;
constexpr uint64_t MIX_M1 = 0x3C6EF372FE9ull;  // odd 43-bit multipliers
constexpr uint64_t MIX_M2 = 0x5851F42D4C9ull;
constexpr int MIX_SHIFT = 22;                   // >= 43/2: x ^= x >> 22 is an involution

constexpr uint64_t inv_odd(uint64_t m) {        // inverse mod 2^64 (Newton), masked to 43 bits later
    uint64_t x = m;
    for (int i = 0; i < 6; ++i) x *= 2 - m * x;
    return x;
}
constexpr uint64_t MIX_I1 = inv_odd(MIX_M1) & KEY_MASK;
constexpr uint64_t MIX_I2 = inv_odd(MIX_M2) & KEY_MASK;

SKM_HD uint64_t mix43(uint64_t k) {
    uint64_t x = (k * MIX_M1) & KEY_MASK;
    x ^= x >> MIX_SHIFT;
    x = (x * MIX_M2) & KEY_MASK;
    x ^= x >> MIX_SHIFT;
    return x;
}
SKM_HD uint64_t unmix43(uint64_t x) {
    x ^= x >> MIX_SHIFT;
    x = (x * MIX_I2) & KEY_MASK;
    x ^= x >> MIX_SHIFT;
    x = (x * MIX_I1) & KEY_MASK;
    return x;
}

// Letters of ok_prot_ relative to 'a': a c d e f g h i k l m n p q r s t v w y
constexpr uint32_t VALID26 = (1u << 0) | (1u << 2) | (1u << 3) | (1u << 4) | (1u << 5) | (1u << 6) |
                             (1u << 7) | (1u << 8) | (1u << 10) | (1u << 11) | (1u << 12) | (1u << 13) |
                             (1u << 15) | (1u << 16) | (1u << 17) | (1u << 18) | (1u << 19) | (1u << 21) |
                             (1u << 22) | (1u << 24);

// code of one residue byte: 0..19 upper-case, 20..39 lower-case, 0xFF if not in ok_prot_.
SKM_HD uint32_t residue_code(uint32_t c) {
    uint32_t idx = (c | 0x20u) - 'a';
    bool valid = idx < 26u && ((VALID26 >> idx) & 1u);
    uint32_t below = VALID26 & ((1u << (idx & 31u)) - 1u);
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t rank = __popc(below);
#else
    uint32_t rank = __builtin_popcount(below);
#endif
    return valid ? rank + ((c & 0x20u) ? 20u : 0u) : 0xFFu;
}

// code -> residue byte.  Arithmetic (no table in memory: on the device a string table costs a
// dependent global byte load per digit): 5-bit offsets from 'A' of ACDEFGHIKLMNPQRSTVWY packed
// 12 + 8 into two constants; codes 20..39 are the lower-case letters.
SKM_HD uint8_t code_residue(uint32_t code) {
    const uint32_t c = code >= 20u ? code - 20u : code;
    const uint64_t w = c < 12u ? 0x6b16a41cc520c40ull : 0xc5ab39460full;
    const uint32_t sh = 5u * (c < 12u ? c : c - 12u);
    return (uint8_t)(65u + (uint32_t)((w >> sh) & 31u) + (code >= 20u ? 32u : 0u));
}

// base-40 code -> little-endian raw key (byte 0 = first residue, the most significant digit).
// Split at 40^4 so the digit loop runs in 32-bit arithmetic.
SKM_HD uint64_t decode_key(uint64_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    // k < 2^43 is exact in fp64; the product can only fall short of an exact multiple of 40^4
    uint64_t q = (uint64_t)((double)k * (1.0 / 2560000.0));
    if (k - q * 2560000u >= 2560000u) ++q;
#else
    const uint64_t q = k / 2560000u;                       // 40^4
#endif
    uint32_t hi4 = (uint32_t)q, lo4 = (uint32_t)(k - q * 2560000u);
    uint64_t raw = 0;
    for (int j = 7; j >= 4; --j) {
        const uint32_t qq = lo4 / 40u;
        raw |= (uint64_t)code_residue(lo4 - qq * 40u) << (8 * j);
        lo4 = qq;
    }
    for (int j = 3; j >= 0; --j) {
        const uint32_t qq = hi4 / 40u;
        raw |= (uint64_t)code_residue(hi4 - qq * 40u) << (8 * j);
        hi4 = qq;
    }
    return raw;
}

// raw little-endian key -> base-40 code (caller guarantees validity)
SKM_HD uint64_t encode_key(uint64_t raw) {
    uint64_t k = 0;
    for (int j = 0; j < 8; ++j) k = k * 40u + residue_code((uint32_t)((raw >> (8 * j)) & 0xFFu));
    return k;
}

// Output slices (skm_build_finish_slice): the kept k-mers whose slice_hash has top bits == slice.
// MurmurHash3's 64-bit finalizer of the little-endian key, independent of the build's own mix43
// so a checker can select the same slice from the raw keys alone.
SKM_HD uint64_t slice_hash(uint64_t key) {
    key ^= key >> 33;
    key *= 0xff51afd7ed558ccdull;
    key ^= key >> 33;
    key *= 0xc4ceb9fe1a85ec53ull;
    key ^= key >> 33;
    return key;
}

// Occurrence record geometry.
struct RecGeom {
    int owner_bits;  // log2(world size)
    int b1_bits;     // level-1 bucket bits
    int rem_bits;    // KEY_BITS - owner_bits - b1_bits
    int pos_bits;    // 64 - rem_bits
};

SKM_HD RecGeom make_geom(int owner_bits, int b1_bits) {
    RecGeom g;
    g.owner_bits = owner_bits;
    g.b1_bits = b1_bits;
    g.rem_bits = KEY_BITS - owner_bits - b1_bits;
    g.pos_bits = 64 - g.rem_bits;
    return g;
}

// LDS element geometry (build, stage 3): lo = s << 36 | i << 16 | offset16
constexpr int ELEM_I_BITS = 20;     // window index within a protein (< 1,048,576 residues)
constexpr int ELEM_S_BITS = 28;     // sequence index within a build (< 268,435,456 sequences)

}  // namespace skm
