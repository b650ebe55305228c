// npow_blake2b.h -- the Nano work hash, specialised for one 40-byte message.
//
// Nano work value (nano-work-server.exe @1660339 blake2b(), @1661643 nano_work;
// server-side rule nanolib.validate_work, server/dpow_server.py:130,365):
//
//   value = LE_u64( BLAKE2b(outlen=8)( LE64(nonce) || root[32] ) )
//
// One compression of one 128-byte block: message words m0 = nonce,
// m1..m4 = root as four little-endian u64, m5..m15 = 0; counter t = 40; final
// block flag set; result = h0 = IV0' ^ v0 ^ v8 where IV0' is the parameter-block
// word IV0 ^ 0x01010008 (digest length 8, fanout 1, depth 1).
//
// This header holds what host and device share: the constants, the sigma
// schedule, and a host (CPU) implementation used for round-1 precomputation,
// CPU re-validation of GPU winners and npow_work_value().  The GPU rounds live
// in npow_kernel.hip and are written on 32-bit halves for the gfx950 VALU.
#pragma once
#include <stdint.h>

namespace npow {

constexpr uint64_t kIV0 = 0x6a09e667f3bcc908ULL, kIV1 = 0xbb67ae8584caa73bULL,
                   kIV2 = 0x3c6ef372fe94f82bULL, kIV3 = 0xa54ff53a5f1d36f1ULL,
                   kIV4 = 0x510e527fade682d1ULL, kIV5 = 0x9b05688c2b3e6c1fULL,
                   kIV6 = 0x1f83d9abfb41bd6bULL, kIV7 = 0x5be0cd19137e2179ULL;

// h0 after the parameter block: IV0 ^ (digest_length=8 | key_length=0 << 8 |
// fanout=1 << 16 | depth=1 << 24)
constexpr uint64_t kH0 = kIV0 ^ 0x01010008ULL;   // 0x6a09e667f2bdc900
constexpr uint64_t kV12 = kIV4 ^ 40ULL;          // t0 = 40 message bytes
constexpr uint64_t kV14 = ~kIV6;                 // final-block flag f0 = ~0

// Message-word schedule for the 12 rounds (rows 10, 11 repeat rows 0, 1).
constexpr uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

// Nonce-independent part of round 1.  Column steps 1..3 of round 1 read only
// m2..m7 (root words 1..3 and zeros), so their outputs are per-root constants
// that the host computes once per task and ships to the kernel as uniform
// (SGPR) arguments.  Column step 0 reads m0 (the nonce) and stays on the GPU.
struct RootPrecomp {
  uint64_t m[4];     // root as 4 LE u64 words (message words m1..m4)
  uint64_t col[12];  // v1,v5,v9,v13, v2,v6,v10,v14, v3,v7,v11,v15 after round-1 columns 1..3
};

inline uint64_t host_load_le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

inline uint64_t host_rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline void host_g(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x, uint64_t y) {
  a = a + b + x;
  d = host_rotr(d ^ a, 32);
  c = c + d;
  b = host_rotr(b ^ c, 24);
  a = a + b + y;
  d = host_rotr(d ^ a, 16);
  c = c + d;
  b = host_rotr(b ^ c, 63);
}

inline void host_init_state(uint64_t v[16]) {
  const uint64_t init[16] = {kH0,  kIV1, kIV2, kIV3, kIV4, kIV5, kIV6, kIV7,
                             kIV0, kIV1, kIV2, kIV3, kV12, kIV5, kV14, kIV7};
  for (int i = 0; i < 16; ++i) v[i] = init[i];
}

inline RootPrecomp host_precompute(const uint8_t root[32]) {
  RootPrecomp p;
  for (int i = 0; i < 4; ++i) p.m[i] = host_load_le64(root + 8 * i);
  uint64_t v[16];
  host_init_state(v);
  // round 1 (sigma row 0): columns 1..3 take m2,m3 | m4,m5 | m6,m7 = h1,h2 | h3,0 | 0,0
  host_g(v[1], v[5], v[9], v[13], p.m[1], p.m[2]);
  host_g(v[2], v[6], v[10], v[14], p.m[3], 0);
  host_g(v[3], v[7], v[11], v[15], 0, 0);
  const int idx[12] = {1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
  for (int i = 0; i < 12; ++i) p.col[i] = v[idx[i]];
  return p;
}

// Full CPU work value (used for re-validation and npow_work_value).
inline uint64_t host_work_value(const uint64_t m_root[4], uint64_t nonce) {
  uint64_t m[16] = {nonce, m_root[0], m_root[1], m_root[2], m_root[3], 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t v[16];
  host_init_state(v);
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = kSigma[r];
    host_g(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
    host_g(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
    host_g(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
    host_g(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
    host_g(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
    host_g(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
    host_g(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
    host_g(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
  }
  return kH0 ^ v[0] ^ v[8];
}

}  // namespace npow
