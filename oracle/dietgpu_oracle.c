/*
 * dietgpu_oracle.c -- serial CPU restatement of the NSagan271/dietgpu_fork
 * rANS byte codec, exponent-split float codec and sparse float codec.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).  The product
 * library (dietgpu_fork_amd/) never links or calls this code.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference/).  Bytes the reference leaves uninitialised ("don't-care",
 * SURVEY.md Appendix B.1) are written as 0 here and by the HIP library.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math: the
 * normalisation's float32 quantisation must round exactly like the GPU).
 */
#define _POSIX_C_SOURCE 200809L
#include "dietgpu_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ans/GpuANSUtils.cuh:33-60 */
#define K_NUM_SYMBOLS 256u
#define K_BLOCK 4096u
#define K_STATE_BITS 31
#define K_ENC_BITS 16
#define K_START_STATE (1u << (K_STATE_BITS - K_ENC_BITS))
#define K_MIN_STATE (1u << (K_STATE_BITS - K_ENC_BITS))
#define K_ANS_MAGIC_VERSION 0xd00d0001u
/* float/GpuFloatUtils.cuh:15-19 */
#define K_FLOAT_MAGIC_VERSION 0xf00f0001u

static uint32_t round_up_u32(uint32_t a, uint32_t b) { return (a + b - 1) / b * b; }
static uint64_t round_up_u64(uint64_t a, uint64_t b) { return (a + b - 1) / b * b; }
static uint32_t div_up_u32(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

static void put32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }
static uint32_t get32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void put16(uint8_t* p, uint16_t v) { memcpy(p, &v, 2); }
static uint16_t get16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }

/* ANSCoalescedHeader::getCompressedOverhead, ans/GpuANSUtils.cuh:68-86:
 * 32 B header + 256 x u16 pdf + 32 x u32 state per block + uint2 per block
 * rounded up to an even count. */
static uint64_t ans_overhead(uint32_t num_blocks) {
  return 32u + 2u * K_NUM_SYMBOLS + 128ull * num_blocks +
         8ull * round_up_u32(num_blocks, 2);
}

/* getMaxCompressedSize, ans/GpuANSEncode.cu:13-25.  Note the reference passes
 * kDefaultBlockSize (4096) as the *block count* to getCompressedOverhead, so
 * the overhead term is the constant 557,600 B; blocks cost
 * getRawCompBlockMaxSize(4096) = 5120 B each (ans/GpuANSEncode.cuh:31-36). */
uint32_t or_max_compressed_size(uint32_t bytes) {
  uint32_t blocks = div_up_u32(bytes, K_BLOCK);
  uint64_t raw = ans_overhead(K_BLOCK);
  raw += (uint64_t)round_up_u32(K_BLOCK + K_BLOCK / 4, 16) * blocks;
  raw = round_up_u64(raw, 16);
  if (raw > 0x7fffffffu) return 0; /* reference CHECK_LE fails */
  return (uint32_t)raw;
}

/* FloatTypeInfo<FT>::getUncompDataSize, float/GpuFloatUtils.cuh:200-391 */
uint32_t or_float_uncomp_data_size(int ft, uint32_t n) {
  switch (ft) {
    case 1: case 2: return round_up_u32(n, 16);
    case 3: return 2 * round_up_u32(n, 8) + round_up_u32(n, 16);
    case 4: return 4 * round_up_u32(n, 4) + 2 * round_up_u32(n, 8);
    default: return 0;
  }
}

static uint32_t word_size(int ft) {
  switch (ft) { case 1: case 2: return 2; case 3: return 4; case 4: return 8; }
  return 0;
}

/* getMaxFloatCompressedSize, float/GpuFloatCompress.cu:23-48 */
uint32_t or_max_float_compressed_size(int ft, uint32_t n) {
  uint32_t base = 32 + or_max_compressed_size(n) + or_float_uncomp_data_size(ft, n);
  if (ft == 4) base += or_max_compressed_size(n);
  return base;
}

/* getMaxSparseFloatCompressedSize, float/GpuSparseFloatCompress.cu:16-24 */
uint32_t or_max_sparse_float_compressed_size(int ft, uint32_t n) {
  return 16 + round_up_u32((n + 7) / 8, 16) + or_max_float_compressed_size(ft, n);
}

/* histogramSingle, ans/GpuANSStatistics.cuh:21-134 (exact counts) */
void or_ans_histogram(const uint8_t* in, size_t n, uint32_t hist[256]) {
  memset(hist, 0, 256 * sizeof(uint32_t));
  for (size_t i = 0; i < n; ++i) hist[in[i]]++;
}

/* checksumSingle, ans/GpuChecksum.cuh:18-93: XOR of all bytes (8-bit). */
uint32_t or_checksum(const uint8_t* in, size_t n) {
  uint32_t c = 0;
  for (size_t i = 0; i < n; ++i) c ^= in[i];
  return c;
}

/* normalizeProbabilitiesFromHistogram, ans/GpuANSStatistics.cuh:178-367,
 * restated for Threads == 256 (one symbol per thread, as quantizeWeights
 * launches it, :414-430). */
int or_ans_normalize(const uint32_t hist[256], uint32_t total, int pb,
                     uint32_t pdf[256], uint32_t cdf[256]) {
  memset(pdf, 0, 256 * sizeof(uint32_t));
  memset(cdf, 0, 256 * sizeof(uint32_t));
  if (total == 0) return 0; /* :193-195 */
  const uint32_t W = 1u << pb;
  uint32_t q[256];
  int qsum = 0;
  for (uint32_t s = 0; s < 256; ++s) {
    /* :212-218 -- uint32 * float -> float, truncated back to uint32 */
    float r = (float)hist[s] / (float)total;
    float f = (float)W * r;
    q[s] = (uint32_t)f;
    if (hist[s] > 0 && q[s] == 0) q[s] = 1;
    qsum += (int)q[s];
  }
  /* :227-243: sort keys (q << 16) | sym descending (unique keys); rank[r] =
   * symbol holding the r-th largest key. */
  int rank_sym[256];
  for (uint32_t s = 0; s < 256; ++s) {
    uint32_t key = (q[s] << 16) | s;
    int r = 0;
    for (uint32_t t = 0; t < 256; ++t) {
      uint32_t kt = (q[t] << 16) | t;
      if (kt > key) ++r;
    }
    rank_sym[r] = (int)s;
  }
  int diff = (int)W - qsum;
  if (diff > 0) {
    /* :258-273: while diff > 0, +1 to every *symbol id* < min(diff, 256) */
    while (diff > 0) {
      int iter = diff < 256 ? diff : 256;
      for (int s = 0; s < iter; ++s) q[s] += 1;
      diff -= iter;
    }
  } else if (diff < 0) {
    /* :274-315: decrement sorted ranks [g-k, g) where g = #{q > 1} */
    int d = -diff;
    while (d > 0) {
      int g = 0;
      for (int s = 0; s < 256; ++s) g += q[s] > 1;
      if (g == 0) return -1; /* reference asserts */
      int k = d < g ? d : g;
      for (int r = g - k; r < g; ++r) q[rank_sym[r]] -= 1;
      d -= k;
    }
  }
  uint32_t run = 0;
  for (int s = 0; s < 256; ++s) { /* :322-341 exclusive scan in symbol order */
    pdf[s] = q[s];
    cdf[s] = run;
    run += q[s];
  }
  return 0;
}

/* ansEncodeWarpBlock + encodeOneWarp/encodeOnePartialWarp,
 * ans/GpuANSEncode.cuh:49-211: 32 interleaved states; symbol t*32+l goes to
 * lane l; emission order within a step = ascending lane among emitting lanes.
 * Returns the number of u16 words written. */
static uint32_t encode_block(const uint8_t* in, uint32_t uw, int pb,
                             const uint32_t* pdf, const uint32_t* cdf,
                             uint32_t states[32], uint16_t* out) {
  uint32_t st[32];
  for (int l = 0; l < 32; ++l) st[l] = K_START_STATE;
  uint32_t nout = 0;
  const uint32_t steps = div_up_u32(uw, 32);
  for (uint32_t t = 0; t < steps; ++t) {
    for (uint32_t l = 0; l < 32; ++l) {
      uint32_t i = t * 32 + l;
      if (i >= uw) continue;
      uint32_t s = in[i];
      uint32_t p = pdf[s];
      uint32_t x = st[l];
      if (x >= (p << (K_STATE_BITS - pb))) { /* :64-75 */
        out[nout++] = (uint16_t)(x & 0xffffu);
        x >>= K_ENC_BITS;
      }
      /* :79-86: ((x / pdf) << pb) + (x % pdf) + cdf */
      x = ((x / p) << pb) + (x % p) + cdf[s];
      st[l] = x;
    }
  }
  for (int l = 0; l < 32; ++l) states[l] = st[l];
  return nout;
}

uint32_t or_ans_encode(const uint8_t* in, uint32_t n, int pb, int use_checksum,
                       const uint32_t* hist_in, uint8_t* out, size_t out_cap) {
  if (pb < 9 || pb > 11) return 0;
  uint32_t hist[256], pdf[256], cdf[256];
  if (hist_in) memcpy(hist, hist_in, sizeof(hist));
  else or_ans_histogram(in, n, hist);
  if (or_ans_normalize(hist, n, pb, pdf, cdf) != 0) return 0;

  const uint32_t nb = div_up_u32(n, K_BLOCK);
  uint32_t* cw = (uint32_t*)calloc(nb ? nb : 1, sizeof(uint32_t));
  uint32_t* pre = (uint32_t*)calloc(nb ? nb : 1, sizeof(uint32_t));
  uint32_t* st = (uint32_t*)calloc((size_t)(nb ? nb : 1) * 32, sizeof(uint32_t));
  /* per-block scratch bounded by 11 bits/symbol + 1 word */
  uint16_t* blk = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(nb ? nb : 1) * 2880);
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t uw = (b + 1 < nb || n % K_BLOCK == 0) ? K_BLOCK : n % K_BLOCK;
    cw[b] = encode_block(in + (size_t)b * K_BLOCK, uw, pb, pdf, cdf,
                         st + (size_t)b * 32, blk + (size_t)b * 2880);
  }
  /* batchExclusivePrefixSum with Align<u16,16>: ans/BatchPrefixSum.cuh,
   * ans/GpuANSEncode.cuh:497-509,785-820 (round each block to 8 words) */
  uint32_t run = 0;
  for (uint32_t b = 0; b < nb; ++b) { pre[b] = run; run += round_up_u32(cw[b], 8); }
  uint32_t total_words = nb ? pre[nb - 1] + round_up_u32(cw[nb - 1], 8) : 0; /* :533-547 */
  uint64_t size = ans_overhead(nb) + 2ull * total_words;
  if (size > out_cap || size > 0xffffffffull) {
    free(cw); free(pre); free(st); free(blk);
    return 0;
  }
  memset(out, 0, (size_t)size);
  /* ansEncodeCoalesce header, ans/GpuANSEncode.cuh:549-573 */
  put32(out + 0, K_ANS_MAGIC_VERSION);
  put32(out + 4, nb);
  put32(out + 8, n);
  put32(out + 12, total_words);
  put32(out + 16, (uint32_t)pb | ((use_checksum ? 1u : 0u) << 4));
  put32(out + 20, use_checksum ? or_checksum(in, n) : 0);
  for (int s = 0; s < 256; ++s) put16(out + 32 + 2 * s, (uint16_t)pdf[s]);
  uint8_t* states = out + 544;
  uint8_t* bwords = states + 128ull * nb;
  uint8_t* data = bwords + 8ull * round_up_u32(nb, 2);
  for (uint32_t b = 0; b < nb; ++b) {
    for (int l = 0; l < 32; ++l) put32(states + 128ull * b + 4 * l, st[(size_t)b * 32 + l]);
    /* :594-604: .x = (uncompressedWords << 16) | compressedWords, .y = prefix */
    uint32_t last = n % K_BLOCK ? n % K_BLOCK : K_BLOCK;
    uint32_t uwb = b == nb - 1 ? last : K_BLOCK;
    put32(bwords + 8ull * b, (uwb << 16) | cw[b]);
    put32(bwords + 8ull * b + 4, pre[b]);
    memcpy(data + 2ull * pre[b], blk + (size_t)b * 2880, 2ull * cw[b]);
  }
  free(cw); free(pre); free(st); free(blk);
  return (uint32_t)size;
}

uint32_t or_ans_info(const uint8_t* a, uint32_t* checksum) {
  if (checksum) *checksum = get32(a + 20);
  return get32(a + 8);
}

uint32_t or_ans_archive_size(const uint8_t* a) {
  uint32_t nb = get32(a + 4);
  return (uint32_t)(ans_overhead(nb) + 2ull * get32(a + 12));
}

/* ansDecodeTable + ansDecodeKernel/ansDecodeWarpBlock,
 * ans/GpuANSDecode.cuh:34-476 */
int or_ans_decode(const uint8_t* a, int pb, int use_checksum, uint8_t* out,
                  uint32_t out_cap, uint32_t* out_size) {
  if (get32(a) != K_ANS_MAGIC_VERSION) return 2;
  uint32_t opts = get32(a + 16);
  if ((int)(opts & 0xf) != pb) return 2;
  const uint32_t nb = get32(a + 4);
  const uint32_t n = get32(a + 8);
  if (out_size) *out_size = n;
  if (out_cap < n) return 1; /* :326-341 capacity check */
  if (n == 0) return 0;
  const uint32_t W = 1u << pb;
  uint32_t pdf[256], cdf[256], run = 0;
  for (int s = 0; s < 256; ++s) { pdf[s] = get16(a + 32 + 2 * s); cdf[s] = run; run += pdf[s]; }
  if (run != W) return 2;
  uint32_t* lut = (uint32_t*)malloc(sizeof(uint32_t) * W);
  for (int s = 0; s < 256; ++s) /* packDecodeLookup :34-44 */
    for (uint32_t j = 0; j < pdf[s]; ++j) lut[cdf[s] + j] = (j << 20) | (pdf[s] << 8) | (uint32_t)s;
  const uint8_t* states = a + 544;
  const uint8_t* bwords = states + 128ull * nb;
  const uint8_t* data = bwords + 8ull * round_up_u32(nb, 2);
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t x[32];
    for (int l = 0; l < 32; ++l) x[l] = get32(states + 128ull * b + 4 * l);
    uint32_t bx = get32(bwords + 8ull * b);
    uint32_t uw = bx >> 16, cwb = bx & 0xffff, start = get32(bwords + 8ull * b + 4);
    const uint8_t* in = data + 2ull * start;
    int64_t ptr = cwb; /* one past the last word */
    uint8_t* ob = out + (size_t)b * K_BLOCK;
    const uint32_t steps = div_up_u32(uw, 32);
    for (int64_t t = (int64_t)steps - 1; t >= 0; --t) {
      /* lanes read in descending lane order: the highest reading lane takes
       * in[ptr-1] (decodeOneWarp :55-105, prefix = popc(vote & lanemask_ge)) */
      for (int l = 31; l >= 0; --l) {
        uint32_t i = (uint32_t)t * 32 + (uint32_t)l;
        if (i >= uw) continue;
        uint32_t e = lut[x[l] & (W - 1)];
        ob[i] = (uint8_t)(e & 0xff);
        x[l] = ((e >> 8) & 0xfff) * (x[l] >> pb) + (e >> 20);
        if (x[l] < K_MIN_STATE) {
          --ptr;
          if (ptr < 0) { free(lut); return 2; }
          x[l] = (x[l] << 16) + get16(in + 2 * ptr);
        }
      }
    }
  }
  free(lut);
  if (use_checksum) {
    /* ansDecodeBatch :557-591; the reference checksums out capacity bytes */
    if (or_checksum(out, out_cap) != get32(a + 20)) return 3;
  }
  return 0;
}

/* ---------------------------- float codec ---------------------------- */

static uint32_t rotl32(uint32_t v, int s) { return (v << s) | (v >> (32 - s)); }
static uint32_t rotr32(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }
static uint64_t rotl64(uint64_t v, int s) { return (v << s) | (v >> (64 - s)); }
static uint64_t rotr64(uint64_t v, int s) { return (v >> s) | (v << (64 - s)); }

/* FloatTypeInfo<FT>::split, float/GpuFloatUtils.cuh:190-370; raw section
 * layout per getUncompDataSize and SplitFloatNonAligned
 * (float/GpuFloatCompress.cuh:168-250). */
static void float_split(int ft, const void* in, uint32_t n, uint8_t* comp0,
                        uint8_t* comp1, uint8_t* raw) {
  if (ft == 1) {
    const uint16_t* w = (const uint16_t*)in;
    for (uint32_t i = 0; i < n; ++i) { comp0[i] = (uint8_t)(w[i] >> 8); raw[i] = (uint8_t)(w[i] & 0xff); }
  } else if (ft == 2) {
    const uint16_t* w = (const uint16_t*)in;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t v = rotl32(((uint32_t)w[i] << 16) | w[i], 1);
      comp0[i] = (uint8_t)(v >> 24);
      raw[i] = (uint8_t)(v & 0xff);
    }
  } else if (ft == 3) {
    const uint32_t* w = (const uint32_t*)in;
    uint8_t* hi = raw + 2 * round_up_u32(n, 8);
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t v = rotl32(w[i], 1);
      comp0[i] = (uint8_t)(v >> 24);
      put16(raw + 2 * i, (uint16_t)(v & 0xffff));
      hi[i] = (uint8_t)((v >> 16) & 0xff);
    }
  } else {
    const uint64_t* w = (const uint64_t*)in;
    uint8_t* hi = raw + 4 * round_up_u32(n, 4);
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t v = rotl64(w[i], 1);
      comp0[i] = (uint8_t)(v >> 56);
      comp1[i] = (uint8_t)((v >> 48) & 0xff);
      put32(raw + 4 * i, (uint32_t)(v & 0xffffffffu));
      put16(hi + 2 * i, (uint16_t)((v >> 32) & 0xffff));
    }
  }
}

/* FloatTypeInfo<FT>::join, float/GpuFloatUtils.cuh:203-367 and
 * JoinFloatNonAligned (float/GpuFloatDecompress.cuh:39-149) */
static void float_join(int ft, const uint8_t* comp0, const uint8_t* comp1,
                       const uint8_t* raw, uint32_t n, void* out) {
  if (ft == 1) {
    uint16_t* w = (uint16_t*)out;
    for (uint32_t i = 0; i < n; ++i) w[i] = (uint16_t)((comp0[i] << 8) | raw[i]);
  } else if (ft == 2) {
    uint16_t* w = (uint16_t*)out;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t lo = (((uint32_t)comp0[i] << 8) | raw[i]) << 16;
      uint32_t hi = raw[i];
      uint32_t v = (lo >> 1) | (hi << 31); /* shf.r.clamp(lo, hi, 1) */
      w[i] = (uint16_t)(v >> 16);
    }
  } else if (ft == 3) {
    uint32_t* w = (uint32_t*)out;
    const uint8_t* hi = raw + 2 * round_up_u32(n, 8);
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t v = ((uint32_t)comp0[i] << 24) | ((uint32_t)hi[i] << 16) | get16(raw + 2 * i);
      w[i] = rotr32(v, 1);
    }
  } else {
    uint64_t* w = (uint64_t*)out;
    const uint8_t* hi = raw + 4 * round_up_u32(n, 4);
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t v = ((uint64_t)comp0[i] << 56) | ((uint64_t)comp1[i] << 48) |
                   ((uint64_t)get16(hi + 2 * i) << 32) | get32(raw + 4 * i);
      w[i] = rotr64(v, 1);
    }
  }
}

/* floatCompressDevice, float/GpuFloatCompress.cuh:670-874: header (16 B),
 * header2 (16 B), raw section, ANS archive #1 of comp bytes (+ #2 for fp64 at
 * roundUp(#1, 16)). */
uint32_t or_float_compress(int ft, const void* in, uint32_t n, int pb,
                           int use_checksum, uint8_t* out, size_t out_cap) {
  if (ft < 1 || ft > 4) return 0;
  const uint32_t rawsz = or_float_uncomp_data_size(ft, n);
  uint8_t* comp0 = (uint8_t*)malloc(n ? n : 1);
  uint8_t* comp1 = (uint8_t*)malloc(n ? n : 1);
  if ((size_t)32 + rawsz > out_cap) { free(comp0); free(comp1); return 0; }
  memset(out, 0, 32 + (size_t)rawsz);
  float_split(ft, in, n, comp0, comp1, out + 32);
  put32(out + 0, K_FLOAT_MAGIC_VERSION);
  put32(out + 4, n);
  put32(out + 8, (uint32_t)ft | ((use_checksum ? 1u : 0u) << 4));
  /* checksumBatch receives the float count as a byte count (Appendix B.3):
   * the checksum covers the first n bytes of the input only. */
  put32(out + 12, use_checksum ? or_checksum((const uint8_t*)in, n) : 0);
  size_t off = 32 + (size_t)rawsz;
  uint32_t a1 = or_ans_encode(comp0, n, pb, 0, NULL, out + off, out_cap - off);
  if (!a1) { free(comp0); free(comp1); return 0; }
  put32(out + 16, round_up_u32(a1, 16)); /* setHeaderAndANSOutOffset :656-667 */
  uint32_t total = 32 + rawsz + a1;
  if (ft == 4) {
    off += round_up_u32(a1, 16);
    uint32_t a2 = or_ans_encode(comp1, n, pb, 0, NULL, out + off, out_cap - off);
    if (!a2) { free(comp0); free(comp1); return 0; }
    total += a2; /* incOutputSizesF64 :570-576 */
  }
  free(comp0); free(comp1);
  return total;
}

int or_float_decompress(const uint8_t* a, int ft, int pb, int use_checksum,
                        void* out, uint32_t cap, uint32_t* out_words) {
  if (get32(a) != K_FLOAT_MAGIC_VERSION) return 2;
  if ((int)(get32(a + 8) & 0xf) != ft) return 2;
  const uint32_t n = get32(a + 4);
  if (out_words) *out_words = n;
  if (cap < n) return 1;
  const uint32_t rawsz = or_float_uncomp_data_size(ft, n);
  uint8_t* comp0 = (uint8_t*)malloc(n ? n : 1);
  uint8_t* comp1 = (uint8_t*)malloc(n ? n : 1);
  uint32_t got = 0;
  const uint8_t* a1 = a + 32 + rawsz;
  int st = or_ans_decode(a1, pb, 0, comp0, n, &got);
  if (st == 0 && ft == 4) st = or_ans_decode(a1 + get32(a + 16), pb, 0, comp1, n, &got);
  if (st == 0 && got != n) st = 2;
  if (st == 0) float_join(ft, comp0, comp1, a + 32, n, out);
  free(comp0); free(comp1);
  if (st) return st;
  if (use_checksum) {
    /* floatDecompressDevice :1077-1112 checksums `capacity` bytes */
    if (or_checksum((const uint8_t*)out, cap) != get32(a + 12)) return 3;
  }
  return 0;
}

/* --------------------------- sparse codec ---------------------------- */

static int word_nonzero(int ft, const void* in, uint32_t i) {
  switch (word_size(ft)) {
    case 2: return ((const uint16_t*)in)[i] != 0;
    case 4: return ((const uint32_t*)in)[i] != 0;
    default: return ((const uint64_t*)in)[i] != 0;
  }
}

/* Compacted nonzero list (float/GpuSparseFloatCompress.cuh:119-185): with
 * idx = exclusive scan of flags, x[i] -> list[idx[i]] for i < n-1 and x[n-1]
 * -> list[idx[n-2] + 1]; count = idx[n-2] + flag[n-1] + 1.  When x[n-2] == 0
 * this leaves one don't-care slot (reference: uninitialised memory; here 0).
 * n == 1: count = flag[0] (reference reads idx[-1]); n == 0: count = 0. */
static uint32_t sparse_compact(int ft, const void* in, uint32_t n, uint8_t* list) {
  const uint32_t ws = word_size(ft);
  if (n == 0) return 0;
  if (n == 1) {
    int f = word_nonzero(ft, in, 0);
    if (f) memcpy(list, in, ws);
    return (uint32_t)f;
  }
  uint32_t idx = 0;
  for (uint32_t i = 0; i + 1 < n; ++i) {
    if (word_nonzero(ft, in, i)) { memcpy(list + (size_t)idx * ws, (const uint8_t*)in + (size_t)i * ws, ws); ++idx; }
  }
  /* idx now = nnz in [0, n-1); idx[n-2] = nnz in [0, n-2) */
  uint32_t idx_nm2 = idx - (uint32_t)word_nonzero(ft, in, n - 2);
  if (!word_nonzero(ft, in, n - 2)) memset(list + (size_t)idx_nm2 * ws, 0, ws);
  int fl = word_nonzero(ft, in, n - 1);
  if (fl) memcpy(list + (size_t)(idx_nm2 + 1) * ws, (const uint8_t*)in + (size_t)(n - 1) * ws, ws);
  return idx_nm2 + (uint32_t)fl + 1;
}

uint32_t or_sparse_float_compress(int ft, const void* in, uint32_t n, int pb,
                                  int use_checksum, uint8_t* out, size_t cap) {
  if (ft < 1 || ft > 4) return 0;
  const uint32_t bm = (n + 7) / 8, bmpad = round_up_u32(bm, 16);
  if ((size_t)16 + bmpad > cap) return 0;
  memset(out, 0, 16 + (size_t)bmpad);
  put32(out, n); /* GpuSparseFloatHeader, float/GpuFloatUtils.cuh:107-124 */
  /* bitmap_bytes_to_bits :64-113: bit 7 of byte k <-> element 8k */
  for (uint32_t i = 0; i < n; ++i)
    if (word_nonzero(ft, in, i)) out[16 + i / 8] |= (uint8_t)(0x80u >> (i % 8));
  uint8_t* list = (uint8_t*)malloc((size_t)(n ? n : 1) * word_size(ft) + 16);
  uint32_t cnt = sparse_compact(ft, in, n, list);
  uint32_t d = or_float_compress(ft, list, cnt, pb, use_checksum, out + 16 + bmpad,
                                 cap - 16 - bmpad);
  free(list);
  if (!d) return 0;
  return 16 + bmpad + d; /* addBitmapToOutSizes :237-247 */
}

int or_sparse_float_decompress(const uint8_t* a, int ft, int pb, int use_checksum,
                               void* out, uint32_t cap, uint32_t* out_words) {
  const uint32_t n = get32(a);
  const uint32_t ws = word_size(ft);
  if (!ws) return 2;
  if (out_words) *out_words = n;
  if (cap < n) return 1;
  const uint32_t bmpad = round_up_u32((n + 7) / 8, 16);
  const uint8_t* dense = a + 16 + bmpad;
  if (get32(dense) != K_FLOAT_MAGIC_VERSION) return 2;
  uint32_t cnt = get32(dense + 4);
  uint8_t* list = (uint8_t*)malloc((size_t)(cnt ? cnt : 1) * ws);
  uint32_t got = 0;
  int st = or_float_decompress(dense, ft, pb, use_checksum, list, cnt, &got);
  if (st) { free(list); return st; }
  /* fill_in_nonzeros, float/GpuSparseFloatDecompress.cuh:69-145 */
  const uint8_t* bmp = a + 16;
  uint32_t idx = 0, idx_nm2 = 0;
  for (uint32_t i = 0; i < n; ++i) {
    int f = (bmp[i / 8] >> (7 - i % 8)) & 1;
    if (i == n - 2) idx_nm2 = idx;
    uint32_t src = idx;
    if (i == n - 1 && n >= 2) src = idx_nm2 + 1;
    uint8_t* dst = (uint8_t*)out + (size_t)i * ws;
    if (f) {
      if (src >= cnt) { free(list); return 2; }
      memcpy(dst, list + (size_t)src * ws, ws);
    } else {
      memset(dst, 0, ws);
    }
    idx += (uint32_t)f;
  }
  free(list);
  return 0;
}

/* ------------------------ CPU baseline timing ------------------------ */

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
  int kind; /* 0 ans, 1 float */
  int ft;
  const uint8_t* in;
  uint32_t units_each; /* bytes (ans) or words (float) */
  size_t stride;
  int pb;
  uint32_t begin, end;
  uint8_t* arch;
  size_t arch_stride;
  uint8_t* dec;
  uint64_t comp;
  int phase; /* 0 encode, 1 decode */
  int fail;
} job_t;

static void* run_job(void* p) {
  job_t* j = (job_t*)p;
  for (uint32_t b = j->begin; b < j->end; ++b) {
    uint8_t* arch = j->arch + (size_t)b * j->arch_stride;
    if (j->phase == 0) {
      uint32_t sz = j->kind == 0
          ? or_ans_encode(j->in + (size_t)b * j->stride, j->units_each, j->pb, 0, NULL, arch, j->arch_stride)
          : or_float_compress(j->ft, j->in + (size_t)b * j->stride, j->units_each, j->pb, 0, arch, j->arch_stride);
      if (!sz) j->fail = 1;
      j->comp += sz;
    } else {
      uint32_t got = 0;
      int st = j->kind == 0
          ? or_ans_decode(arch, j->pb, 0, j->dec, j->units_each, &got)
          : or_float_decompress(arch, j->ft, j->pb, 0, j->dec, j->units_each, &got);
      if (st) j->fail = 1;
    }
  }
  return NULL;
}

static double time_roundtrip(int kind, int ft, const uint8_t* in, uint32_t nb,
                             uint32_t units, size_t stride, int pb, int threads,
                             uint64_t* comp_total, double* enc_s, double* dec_s) {
  size_t arch_stride = kind == 0 ? or_max_compressed_size(units)
                                 : or_max_float_compressed_size(ft, units);
  size_t dec_bytes = kind == 0 ? units : (size_t)units * word_size(ft);
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > nb) threads = (int)(nb ? nb : 1);
  uint8_t* arch = (uint8_t*)malloc(arch_stride * (nb ? nb : 1));
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  double t[3];
  int fail = 0;
  uint64_t comp = 0;
  for (int phase = 0; phase < 2; ++phase) {
    for (int k = 0; k < threads; ++k) {
      job_t* j = &jobs[k];
      j->kind = kind; j->ft = ft; j->in = in; j->units_each = units; j->stride = stride;
      j->pb = pb; j->begin = (uint32_t)((uint64_t)nb * k / threads);
      j->end = (uint32_t)((uint64_t)nb * (k + 1) / threads);
      j->arch = arch; j->arch_stride = arch_stride; j->phase = phase;
      if (phase == 0) { j->comp = 0; j->fail = 0; j->dec = NULL; }
      else if (!j->dec) j->dec = (uint8_t*)malloc(dec_bytes ? dec_bytes : 1);
    }
    t[phase] = now_s();
    if (threads == 1) run_job(&jobs[0]);
    else {
      for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, run_job, &jobs[k]);
      for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    }
    t[phase + 1] = now_s();
  }
  for (int k = 0; k < threads; ++k) { comp += jobs[k].comp; fail |= jobs[k].fail; free(jobs[k].dec); }
  free(arch); free(jobs); free(th);
  if (comp_total) *comp_total = comp;
  if (enc_s) *enc_s = t[1] - t[0];
  if (dec_s) *dec_s = t[2] - t[1];
  return fail ? -1.0 : (t[2] - t[0]);
}

double or_time_float_roundtrip(int ft, const void* in, uint32_t nb, uint32_t words,
                               size_t stride, int pb, int threads, uint64_t* comp,
                               double* enc_s, double* dec_s) {
  return time_roundtrip(1, ft, (const uint8_t*)in, nb, words, stride, pb, threads, comp, enc_s, dec_s);
}

double or_time_ans_roundtrip(const uint8_t* in, uint32_t nb, uint32_t bytes,
                             size_t stride, int pb, int threads, uint64_t* comp,
                             double* enc_s, double* dec_s) {
  return time_roundtrip(0, 0, in, nb, bytes, stride, pb, threads, comp, enc_s, dec_s);
}
