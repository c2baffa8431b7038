// kma_pack.cpp — host packing of ASCII residues into the packed residue stream of the protein
// kernel (kma_device.h: residue j = the 5-bit code at bits [5j, 5j + 5) of a big-endian bit
// stream; 8 residues = 5 bytes). Host entry points pack while they stage a batch, so the H2D
// moves 0.625 bytes per residue instead of 1. Plain C++ (host only); an AVX2 path when the CPU
// has it, chosen at run time.
#include "kma_pack.h"

#include <cstdint>
#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace kma {
namespace {

// Eight residues -> five stream bytes (first residue in the most significant bits).
inline void pack8_scalar(const uint8_t* lut, const uint8_t* in, uint8_t* out) {
  uint64_t v = 0;
  for (int j = 0; j < 8; ++j) v = (v << 5) | lut[in[j]];
  for (int b = 0; b < 5; ++b) out[b] = (uint8_t)(v >> (32 - 8 * b));
}

void pack_scalar(const uint8_t* lut, const uint8_t* in, uint64_t n8, uint8_t* out) {
  for (uint64_t g = 0; g < n8; ++g) pack8_scalar(lut, in + 8 * g, out + 5 * g);
}

#if defined(__x86_64__)
// 32 residues (four groups of 8) per step: codes by compares (the table LUT is the standard
// alphabet 'A'..'Z' -> 1..26, '*' -> 27, plus up to four extra bytes -> 28..31), then
// maddubs / madd fold 8 codes into 40 bits per 64-bit lane, and a byte shuffle puts each
// lane's 5 bytes most significant first (two 10-byte halves per step).
struct Avx2Packer {
  __m256i k64, k91, star, c27, w5, w10, m40, shuf, ex[4], ec[4];
  int n_extra;
  __attribute__((target("avx2"))) Avx2Packer(const uint8_t* extra, int n) : n_extra(n) {
    k64 = _mm256_set1_epi8(64);
    k91 = _mm256_set1_epi8(91);
    star = _mm256_set1_epi8('*');
    c27 = _mm256_set1_epi8(27);
    w5 = _mm256_set1_epi16(0x0120);       // bytes (32, 1): c0 * 32 + c1
    w10 = _mm256_set1_epi32(0x00010400);  // words (1024, 1)
    m40 = _mm256_set1_epi64x(0xFFFFFFFFFFll);
    shuf = _mm256_setr_epi8(4, 3, 2, 1, 0, 12, 11, 10, 9, 8, -1, -1, -1, -1, -1, -1,
                            4, 3, 2, 1, 0, 12, 11, 10, 9, 8, -1, -1, -1, -1, -1, -1);
    for (int i = 0; i < n; ++i) {
      ex[i] = _mm256_set1_epi8((char)extra[i]);
      ec[i] = _mm256_set1_epi8((char)(28 + i));
    }
  }
  // 32 residues -> two 10-byte halves in the low 10 bytes of each 128-bit lane
  __attribute__((target("avx2"))) __m256i step(const uint8_t* in) const {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in));
    // 'A'..'Z': 64 < x < 91 as signed bytes (bytes >= 128 are negative: no code)
    const __m256i az = _mm256_and_si256(_mm256_cmpgt_epi8(x, k64), _mm256_cmpgt_epi8(k91, x));
    __m256i c = _mm256_and_si256(az, _mm256_sub_epi8(x, k64));
    c = _mm256_or_si256(c, _mm256_and_si256(_mm256_cmpeq_epi8(x, star), c27));
    for (int i = 0; i < n_extra; ++i)
      c = _mm256_or_si256(c, _mm256_and_si256(_mm256_cmpeq_epi8(x, ex[i]), ec[i]));
    const __m256i t16 = _mm256_maddubs_epi16(c, w5);    // 10-bit pairs
    const __m256i t32 = _mm256_madd_epi16(t16, w10);    // 20-bit quads
    const __m256i v = _mm256_or_si256(_mm256_and_si256(_mm256_slli_epi64(t32, 20), m40),
                                      _mm256_srli_epi64(t32, 32));  // 40 bits per lane
    return _mm256_shuffle_epi8(v, shuf);
  }
};

// n32 steps of 32 residues, 20 output bytes each (two overlapping 16-byte stores: each writes
// 6 bytes past its 10, overwritten by the next; the caller keeps 6 bytes of room after the last)
__attribute__((target("avx2"))) void pack_avx2(const Avx2Packer& p, const uint8_t* in,
                                              uint64_t n32, uint8_t* out) {
  for (uint64_t s = 0; s < n32; ++s) {
    const __m256i b = p.step(in + 32 * s);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 20 * s), _mm256_castsi256_si128(b));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 20 * s + 10), _mm256_extracti128_si256(b, 1));
  }
}

// n512 blocks of 512 residues into a 64-byte aligned `out`, 320 bytes (five lines) each:
// assembled in a stack buffer, then written with non-temporal stores. A staging buffer that
// is only written here and read by the DMA engine then costs no read for ownership of its
// lines: plain stores read every destination line first, 194 MB of extra host-memory reads
// for c5's packed stream, on the same memory the packing reads and the copies drain.
__attribute__((target("avx2"))) void pack_avx2_stream(const Avx2Packer& p, const uint8_t* in,
                                                     uint64_t n512, uint8_t* out) {
  alignas(64) uint8_t buf[320 + 32];
  for (uint64_t blk = 0; blk < n512; ++blk) {
    for (int s = 0; s < 16; ++s) {
      const __m256i b = p.step(in + 512 * blk + 32 * s);
      _mm_storeu_si128(reinterpret_cast<__m128i*>(buf + 20 * s), _mm256_castsi256_si128(b));
      _mm_storeu_si128(reinterpret_cast<__m128i*>(buf + 20 * s + 10), _mm256_extracti128_si256(b, 1));
    }
    for (int i = 0; i < 10; ++i)
      _mm256_stream_si256(reinterpret_cast<__m256i*>(out + 320 * blk + 32 * i),
                          _mm256_load_si256(reinterpret_cast<const __m256i*>(buf + 32 * i)));
  }
  _mm_sfence();  // the stores are visible before the caller publishes the chunk
}
#endif

}  // namespace

void pack_residues_host(const uint8_t lut[256], const uint8_t* in, uint64_t n, uint8_t* out,
                        uint64_t out_cap) {
  const uint64_t whole8 = n / 8;
  uint64_t done8 = 0;
#if defined(__x86_64__)
  static const bool avx2 = __builtin_cpu_supports("avx2");
  uint8_t extra[4];
  int n_extra = 0;
  bool standard = lut[0] == 0;
  for (int c = 0; c < 256 && standard; ++c) {
    const uint8_t v = lut[c];
    if (c >= 'A' && c <= 'Z') standard = v == c - 'A' + 1;
    else if (c == '*') standard = v == 27;
    else if (v >= 28 && v <= 31 && n_extra < 4 && v == 28 + n_extra) extra[n_extra++] = (uint8_t)c;
    else standard = v == 0;
  }
  if (avx2 && standard && whole8 >= 8) {
    const Avx2Packer p(extra, n_extra);
    if (((uintptr_t)out & 63) == 0) {  // whole 512-residue blocks by non-temporal stores
      const uint64_t n512 = whole8 / 64;
      pack_avx2_stream(p, in, n512, out);
      done8 = 64 * n512;
    }
    // the overlapping stores write 6 bytes past their 20: keep the last step for the scalar loop
    if (whole8 - done8 >= 8) {
      const uint64_t n32 = (whole8 - done8 - 4) / 4;
      pack_avx2(p, in + 8 * done8, n32, out + 5 * done8);
      done8 += 4 * n32;
    }
  }
#endif
  pack_scalar(lut, in + 8 * done8, whole8 - done8, out + 5 * done8);
  uint8_t tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t o = 5 * whole8;
  if (n % 8) {
    std::memcpy(tail, in + 8 * whole8, n % 8);  // past n: byte 0 (no code)
    pack8_scalar(lut, tail, out + o);
    o += 5;
  }
  if (out_cap > o) std::memset(out + o, 0, out_cap - o);  // padding the kernel reads
}

}  // namespace kma
