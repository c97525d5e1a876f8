/*
 * oracle.c -- single-threaded C restatement of the reference CPU path.
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the checker for the
 * full-size on-box parity tests and the bench's cpu_baseline ("port").
 *
 * It follows the reference loops, not the GPU design:
 *   - Polynomial::ntt / LagrangePolynomial::intt (src/ntt/mod.rs:69-173):
 *     clone, bit_reverse_permutation, unrolled len=2 stage, iterative DIT with
 *     a serial per-stage twiddle vector gen^(n/len) powers, n^-1 scaling;
 *   - NttField::pow_2_generator_powers (src/ntt/mod.rs:18-28), serial;
 *   - reed_solomon (src/fri/mod.rs:19-28): resize to 2N, ntt;
 *   - commit_rs_code + Merkle::commit (src/fri/mod.rs:45-55,
 *     src/merkle_tree/mod.rs:65-85, :178-189): SHA-256 leaves of the 32-byte
 *     pairs, chunks(2) levels, all layers kept;
 *   - FriProverData::fold_step / fold (src/fri/mod.rs:79-145): clone of the
 *     layer, twiddle gen_pows[len - i*2^k], multiply by half;
 *   - Transcript (src/transcript.rs): running SHA-256;
 *   - to_coefficient (src/polynomials.rs:150-163), Mask-based delta table
 *     (sumcheck.rs:128-145, evaluation.rs:51-73), partial_sum / fold
 *     (sumcheck.rs:204-247).
 * Field: M = 2^128 - 45*2^40 + 1, canonical u128 little endian.
 * SHA-256: FIPS 180-4, written here (the reference uses the sha2 crate).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

static const u128 MOD = (((u128)0xFFFFFFFFFFFFFFFFull) << 64) | (u128)0xFFFFD30000000001ull;
static const uint64_t CF = 0x2CFFFFFFFFFFull; /* 2^128 mod M */

static inline u128 fadd(u128 a, u128 b) {
  u128 s = a + b;
  if (s < a) return s + CF; /* wrapped past 2^128 */
  return s >= MOD ? s - MOD : s;
}
static inline u128 fsub(u128 a, u128 b) { return a >= b ? a - b : a - b + MOD; }

/* 128x128 -> 256, then fold hi*2^128 = hi*CF until hi = 0 */
static inline u128 fmul(u128 a, u128 b) {
  uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  /* column accumulate into 4 x 64-bit words */
  uint64_t w0 = (uint64_t)p00;
  u128 t = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  uint64_t w1 = (uint64_t)t;
  t = (t >> 64) + (p01 >> 64) + (p10 >> 64) + (uint64_t)p11;
  uint64_t w2 = (uint64_t)t;
  uint64_t w3 = (uint64_t)((t >> 64) + (p11 >> 64));
  u128 lo = ((u128)w1 << 64) | w0;
  u128 hi = ((u128)w3 << 64) | w2;
  while (hi) {
    /* hi * CF: hi < 2^128, CF < 2^46 */
    uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
    u128 q0 = (u128)h0 * CF; /* < 2^110 */
    u128 q1 = (u128)h1 * CF; /* < 2^110, weight 2^64 */
    u128 nhi = q1 >> 64;
    u128 add1 = q1 << 64;
    u128 s = lo + q0;
    if (s < lo) nhi++;
    u128 s2 = s + add1;
    if (s2 < s) nhi++;
    lo = s2;
    hi = nhi;
  }
  return lo >= MOD ? lo - MOD : lo;
}
static u128 fpow(u128 b, u128 e) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = fmul(r, b);
    b = fmul(b, b);
    e >>= 1;
  }
  return r;
}
static u128 finv(u128 a) { return fpow(a, MOD - 2); }

static inline u128 ld(const uint8_t* p) {
  u128 v;
  memcpy(&v, p, 16);
  return v;
}
static inline void st(uint8_t* p, u128 v) { memcpy(p, &v, 16); }

/* ------------------------------------------------------------------ SHA-256 */
typedef struct {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len;
} sha_t;

static const uint32_t SK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_block(uint32_t h[8], const uint8_t* b) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) |
           ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = bb;
    bb = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += bb;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

static void sha_init(sha_t* s) {
  static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  memcpy(s->h, iv, 32);
  s->len = 0;
}
static void sha_update(sha_t* s, const uint8_t* p, size_t n) {
  while (n) {
    size_t fill = s->len % 64, take = 64 - fill < n ? 64 - fill : n;
    memcpy(s->buf + fill, p, take);
    s->len += take;
    p += take;
    n -= take;
    if (s->len % 64 == 0) sha_block(s->h, s->buf);
  }
}
static void sha_final(const sha_t* s0, uint8_t out[32]) {
  sha_t s = *s0;
  uint64_t bits = s.len * 8;
  uint8_t one = 0x80, zero = 0;
  sha_update(&s, &one, 1);
  while (s.len % 64 != 56) sha_update(&s, &zero, 1);
  uint8_t lb[8];
  for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(&s, lb, 8);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = s.h[i] >> 24;
    out[4 * i + 1] = s.h[i] >> 16;
    out[4 * i + 2] = s.h[i] >> 8;
    out[4 * i + 3] = s.h[i];
  }
}
void orc_sha256(const uint8_t* msg, uint64_t len, uint8_t out[32]) {
  sha_t s;
  sha_init(&s);
  sha_update(&s, msg, len);
  sha_final(&s, out);
}

/* ---------------------------------------------------------------------- NTT */
static uint64_t rev_bits(uint64_t x, int bits) {
  uint64_t r = 0;
  for (int b = 0; b < bits; b++) r |= ((x >> b) & 1ull) << (bits - 1 - b);
  return r;
}

static void bit_reverse_permutation(u128* v, uint64_t n) {
  int bits = 0;
  while ((1ull << bits) < n) bits++;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t j = rev_bits(i, bits);
    if (i < j) {
      u128 t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
}

static void dit(u128* v, uint64_t n, u128 gen) {
  for (uint64_t i = 0; i < n; i += 2) {
    u128 u = v[i], w = v[i + 1];
    v[i] = fadd(u, w);
    v[i + 1] = fsub(u, w);
  }
  u128* pows = (u128*)malloc(sizeof(u128) * (n / 2 > 0 ? n / 2 : 1));
  for (uint64_t len = 4; len <= n; len *= 2) {
    u128 cur = fpow(gen, n / len), acc = 1;
    for (uint64_t j = 0; j < len / 2; j++) {
      pows[j] = acc;
      acc = fmul(acc, cur);
    }
    for (uint64_t i = 0; i < n; i += len)
      for (uint64_t j = 0; j < len / 2; j++) {
        u128 w = fmul(v[i + j + len / 2], pows[j]), u = v[i + j];
        v[i + j] = fadd(u, w);
        v[i + j + len / 2] = fsub(u, w);
      }
  }
  free(pows);
}

/* in/out: 2^log_n elements (16 B each); may alias. */
int orc_ntt(const uint8_t* in, uint8_t* out, uint32_t log_n, const uint8_t gen[16], int inverse) {
  uint64_t n = 1ull << log_n;
  if (log_n < 1) return 2;
  u128* v = (u128*)malloc(n * sizeof(u128));
  if (!v) return 5;
  memcpy(v, in, n * 16); /* clone (ntt/mod.rs:76) */
  bit_reverse_permutation(v, n);
  u128 g = ld(gen);
  if (inverse) g = finv(g);
  dit(v, n, g);
  if (inverse) {
    u128 ninv = finv((u128)n);
    for (uint64_t i = 0; i < n; i++) v[i] = fmul(v[i], ninv);
  }
  memcpy(out, v, n * 16);
  free(v);
  return 0;
}


/* OpenMP variant of orc_ntt (same loops, butterflies of a stage split over
 * `threads` cores; twiddle table of each stage built in per-thread chunks).
 * The cpu_baseline "all host cores" figure; not a checker. */
#ifdef _OPENMP
#include <omp.h>
#endif
int orc_ntt_omp(const uint8_t* in, uint8_t* out, uint32_t log_n, const uint8_t gen[16], int threads) {
  uint64_t n = 1ull << log_n;
  if (log_n < 1) return 2;
  u128* v = (u128*)malloc(n * sizeof(u128));
  u128* pows = (u128*)malloc(sizeof(u128) * (n / 2));
  if (!v || !pows) return 5;
  memcpy(v, in, n * 16);
  int bits = (int)log_n;
  long long N = (long long)n;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long i = 0; i < N; i++) {
    uint64_t j = rev_bits((uint64_t)i, bits);
    if ((uint64_t)i < j) {
      u128 t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
  u128 g = ld(gen);
  for (uint64_t len = 2; len <= n; len *= 2) {
    const u128 cur = fpow(g, n / len);
    const long long half = (long long)(len / 2);
#pragma omp parallel num_threads(threads)
    {
#ifdef _OPENMP
      const int t = omp_get_thread_num(), T = omp_get_num_threads();
#else
      const int t = 0, T = 1;
#endif
      const long long lo = half * t / T, hi = half * (t + 1) / T;
      u128 acc = fpow(cur, (u128)lo);
      for (long long j = lo; j < hi; j++) {
        pows[j] = acc;
        acc = fmul(acc, cur);
      }
    }
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long b = 0; b < N / 2; b++) {
      const uint64_t i = ((uint64_t)b / half) * len, j = (uint64_t)b % half;
      u128 w = fmul(v[i + j + half], pows[j]), u = v[i + j];
      v[i + j] = fadd(u, w);
      v[i + j + half] = fsub(u, w);
    }
  }
  memcpy(out, v, n * 16);
  free(v);
  free(pows);
  return 0;
}

void orc_pow_2_generator(uint32_t log_size, uint8_t out[16]) {
  st(out, fpow(3, (MOD - 1) >> log_size));
}

void orc_pow_2_generator_powers(uint32_t log_size, uint8_t* out) {
  u128 g = fpow(3, (MOD - 1) >> log_size), cur = 1;
  for (uint64_t i = 0; i < (1ull << log_size); i++) {
    st(out + 16 * i, cur);
    cur = fmul(cur, g);
  }
}

int orc_reed_solomon(const uint8_t* coeffs, uint32_t log_n, const uint8_t gen[16], uint8_t* code) {
  uint64_t n = 1ull << log_n;
  uint8_t* tmp = (uint8_t*)calloc(2 * n, 16);
  memcpy(tmp, coeffs, n * 16);
  int r = orc_ntt(tmp, code, log_n + 1, gen, 0);
  free(tmp);
  return r;
}

/* ------------------------------------------------------------------- Merkle */
/* layers: (2L-1)*32 bytes, leaves first; pairs (code[i], code[i + n/2]). */
void orc_merkle_commit_pairs(const uint8_t* code, uint32_t log_code, uint8_t* layers) {
  uint64_t n = 1ull << log_code, L = n / 2;
  for (uint64_t i = 0; i < L; i++) {
    uint8_t leaf[32];
    memcpy(leaf, code + 16 * i, 16);
    memcpy(leaf + 16, code + 16 * (i + L), 16);
    orc_sha256(leaf, 32, layers + 32 * i);
  }
  uint64_t off = 0, cnt = L;
  while (cnt > 1) {
    for (uint64_t j = 0; j < cnt / 2; j++)
      orc_sha256(layers + 32 * (off + 2 * j), 64, layers + 32 * (off + cnt + j));
    off += cnt;
    cnt /= 2;
  }
}

/* ------------------------------------------------------------------ FRI fold */
/* FriProverData::fold with a fresh transcript (fri/mod.rs:136-145): writes the
 * T = log_code - 1 roots and the last element; returns 6 if not an RS code. */
int orc_fri_commit(const uint8_t* code, uint32_t log_code, uint8_t* roots, uint8_t last[16],
                   uint8_t last_random[32]) {
  uint64_t n0 = 1ull << log_code;
  sha_t tr;
  sha_init(&tr);
  u128 g = fpow(3, (MOD - 1) >> log_code);
  u128 ginv = finv(g), inv2 = finv(2);
  /* gen_pows (ntt/mod.rs:18-28), used as gen_pows[len - i*2^k] */
  u128* gp = (u128*)malloc(n0 * sizeof(u128));
  u128 cur = 1;
  for (uint64_t i = 0; i < n0; i++) {
    gp[i] = cur;
    cur = fmul(cur, g);
  }
  (void)ginv;
  u128* layer = (u128*)malloc(n0 * sizeof(u128));
  memcpy(layer, code, n0 * 16);
  uint8_t* tree = (uint8_t*)malloc((n0 - 1) * 32);
  uint64_t n = n0;
  uint32_t t = 0;
  orc_merkle_commit_pairs((const uint8_t*)layer, log_code, tree);
  memcpy(roots + 32 * t, tree + 32 * (n - 2), 32);
  sha_update(&tr, roots + 32 * t, 32);
  t++;
  int rc = 0;
  for (uint32_t k = 0; k + 1 < log_code; k++) {
    uint8_t rnd[32];
    sha_final(&tr, rnd);
    u128 r = ld(rnd);
    if (r >= MOD) r -= MOD;
    uint64_t half = n / 2;
    u128* next = (u128*)malloc(half * sizeof(u128)); /* clone + fold */
    for (uint64_t i = 0; i < half; i++) {
      u128 a = layer[i], b = layer[i + half];
      u128 tw = i == 0 ? 1 : gp[n0 - i * (1ull << k)];
      u128 odd = fmul(fsub(a, b), tw);
      next[i] = fmul(fadd(fadd(a, b), fmul(r, odd)), inv2);
    }
    free(layer);
    layer = next;
    n = half;
    if (half == 2) {
      if (layer[0] != layer[1]) rc = 6;
      st(last, layer[0]);
      sha_update(&tr, last, 16);
      break;
    }
    orc_merkle_commit_pairs((const uint8_t*)layer, (uint32_t)__builtin_ctzll(n), tree);
    memcpy(roots + 32 * t, tree + 32 * (n - 2), 32);
    sha_update(&tr, roots + 32 * t, 32);
    t++;
  }
  if (last_random) sha_final(&tr, last_random);
  free(layer);
  free(tree);
  free(gp);
  return rc;
}

/* ------------------------------------------------------- multilinear / sumcheck */
void orc_to_coefficient(uint8_t* v, uint32_t log_n) {
  uint64_t n = 1ull << log_n;
  for (uint32_t i = 0; i < log_n; i++) {
    uint64_t m = 1ull << i;
    for (uint64_t j = 0; j < n; j++)
      if (j & m) st(v + 16 * j, fsub(ld(v + 16 * j), ld(v + 16 * (j ^ m))));
  }
}

/* delta[idx] = prod_i (bit_i(idx) ? p[n-1-i] : 1 - p[n-1-i]) -- n mults per entry */
void orc_eq_table(const uint8_t* pts, uint32_t n, uint8_t* out) {
  for (uint64_t idx = 0; idx < (1ull << n); idx++) {
    u128 acc = 1;
    for (uint32_t i = 0; i < n; i++) {
      u128 p = ld(pts + 16 * (n - 1 - i));
      acc = fmul(acc, ((idx >> i) & 1) ? p : fsub(1, p));
    }
    st(out + 16 * idx, acc);
  }
}

/* partial_sum at X=1 and X=2 (sumcheck.rs:204-232), composition x[0]. */
void orc_partial_sums(const uint8_t* m, const uint8_t* d, uint32_t log_h, uint8_t out[32]) {
  uint64_t off = (1ull << log_h) / 2;
  u128 s1 = 0, s2 = 0;
  for (uint64_t i = 0; i < off; i++) s1 = fadd(s1, fmul(ld(m + 16 * (i + off)), ld(d + 16 * (i + off))));
  u128 r = 2, s = fsub(1, r);
  for (uint64_t i = 0; i < off; i++) {
    u128 dd = fadd(fmul(s, ld(d + 16 * i)), fmul(r, ld(d + 16 * (i + off))));
    u128 mm = fadd(fmul(s, ld(m + 16 * i)), fmul(r, ld(m + 16 * (i + off))));
    s2 = fadd(s2, fmul(mm, dd));
  }
  st(out, s1);
  st(out + 16, s2);
}

/* fold (sumcheck.rs:234-247), in place */
void orc_fold(uint8_t* m, uint8_t* d, uint32_t log_h, const uint8_t rb[16]) {
  uint64_t off = (1ull << log_h) / 2;
  u128 r = ld(rb), s = fsub(1, r);
  for (uint64_t i = 0; i < off; i++) {
    st(d + 16 * i, fadd(fmul(s, ld(d + 16 * i)), fmul(r, ld(d + 16 * (i + off)))));
    st(m + 16 * i, fadd(fmul(s, ld(m + 16 * i)), fmul(r, ld(m + 16 * (i + off)))));
  }
}

/* field op KATs for the tests */
void orc_mul(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]) {
  st(out, fmul(ld(a), ld(b)));
}

/* ------------------------------------------------------- parallel checkers */
/* The same arithmetic with OpenMP over independent work (butterflies of a
 * stage, leaves/nodes of a Merkle level, entries of the eq table, pairs of a
 * fold).  Field results are exact, so they equal the serial restatement; these
 * exist only so the full-size parity tests (config 3 at 2^25, config 4 at 24
 * variables, config 5 at 2^28) finish within a test's time limit on the GPU
 * box's host cores.  Not a baseline. */
static void pow_series_par(u128* pw, uint64_t count, u128 g, int threads) {
#pragma omp parallel num_threads(threads)
  {
#ifdef _OPENMP
    const int t = omp_get_thread_num(), T = omp_get_num_threads();
#else
    const int t = 0, T = 1;
#endif
    const uint64_t lo = count * (uint64_t)t / (uint64_t)T, hi = count * (uint64_t)(t + 1) / (uint64_t)T;
    u128 acc = fpow(g, (u128)lo);
    for (uint64_t j = lo; j < hi; j++) {
      pw[j] = acc;
      acc = fmul(acc, g);
    }
  }
}

int orc_ntt_par(const uint8_t* in, uint8_t* out, uint32_t log_n, const uint8_t gen[16], int inverse,
                int threads) {
  const uint64_t n = 1ull << log_n;
  if (log_n < 1) return 2;
  u128* v = (u128*)malloc(n * sizeof(u128));
  u128* pw = (u128*)malloc((n / 2) * sizeof(u128));
  if (!v || !pw) return 5;
  memcpy(v, in, n * 16);
  const long long N = (long long)n;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long i = 0; i < N; i++) {
    const uint64_t j = rev_bits((uint64_t)i, (int)log_n);
    if ((uint64_t)i < j) {
      u128 t = v[i];
      v[i] = v[j];
      v[j] = t;
    }
  }
  u128 g = ld(gen);
  if (inverse) g = finv(g);
  pow_series_par(pw, n / 2, g, threads);  /* stage len: twiddle j = g^(j n/len) */
  const uint64_t B = n < (1ull << 14) ? n : (1ull << 14);
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long b = 0; b < (long long)(n / B); b++) {
    u128* blk = v + (uint64_t)b * B;
    for (uint64_t len = 2; len <= B; len *= 2)
      for (uint64_t i = 0; i < B; i += len)
        for (uint64_t j = 0; j < len / 2; j++) {
          const u128 w = fmul(blk[i + j + len / 2], pw[j * (n / len)]), u = blk[i + j];
          blk[i + j] = fadd(u, w);
          blk[i + j + len / 2] = fsub(u, w);
        }
  }
  for (uint64_t len = 2 * B; len <= n; len *= 2) {
    const long long half = (long long)(len / 2);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long q = 0; q < N / 2; q++) {
      const uint64_t i = ((uint64_t)q / half) * len, j = (uint64_t)q % half;
      const u128 w = fmul(v[i + j + half], pw[j * (n / len)]), u = v[i + j];
      v[i + j] = fadd(u, w);
      v[i + j + half] = fsub(u, w);
    }
  }
  if (inverse) {
    const u128 ninv = finv((u128)n);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long i = 0; i < N; i++) v[i] = fmul(v[i], ninv);
  }
  memcpy(out, v, n * 16);
  free(v);
  free(pw);
  return 0;
}

int orc_reed_solomon_par(const uint8_t* coeffs, uint32_t log_n, const uint8_t gen[16], uint8_t* code,
                         int threads) {
  const uint64_t n = 1ull << log_n;
  uint8_t* tmp = (uint8_t*)calloc(2 * n, 16);
  if (!tmp) return 5;
  memcpy(tmp, coeffs, n * 16);
  const int r = orc_ntt_par(tmp, code, log_n + 1, gen, 0, threads);
  free(tmp);
  return r;
}

static void merkle_pairs_par(const uint8_t* code, uint32_t log_code, uint8_t* layers, int threads) {
  const uint64_t n = 1ull << log_code, L = n / 2;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long i = 0; i < (long long)L; i++) {
    uint8_t leaf[32];
    memcpy(leaf, code + 16 * (uint64_t)i, 16);
    memcpy(leaf + 16, code + 16 * ((uint64_t)i + L), 16);
    orc_sha256(leaf, 32, layers + 32 * (uint64_t)i);
  }
  uint64_t off = 0, cnt = L;
  while (cnt > 1) {
#pragma omp parallel for num_threads(threads) schedule(static) if (cnt > 4096)
    for (long long j = 0; j < (long long)(cnt / 2); j++)
      orc_sha256(layers + 32 * (off + 2 * (uint64_t)j), 64, layers + 32 * (off + cnt + (uint64_t)j));
    off += cnt;
    cnt /= 2;
  }
}

/* orc_fri_commit with the work of each layer in parallel; gen_pows has
 * 2^log_gp >= 2^log_code entries of the order-2^log_gp generator (the
 * reference's fold twiddle is gen_pows[len - i 2^k], len = gen_pows.len()). */
int orc_fri_commit_par(const uint8_t* code, uint32_t log_code, uint32_t log_gp, uint8_t* roots,
                       uint8_t last[16], uint8_t last_random[32], int threads) {
  const uint64_t n0 = 1ull << log_code, glen = 1ull << log_gp;
  if (log_gp < log_code) return 2;
  sha_t tr;
  sha_init(&tr);
  const u128 g = fpow(3, (MOD - 1) >> log_gp), inv2 = finv(2);
  u128* gp = (u128*)malloc(glen * sizeof(u128));
  u128* layer = (u128*)malloc(n0 * sizeof(u128));
  u128* next = (u128*)malloc((n0 / 2) * sizeof(u128));
  uint8_t* tree = (uint8_t*)malloc((n0 - 1) * 32);
  if (!gp || !layer || !next || !tree) return 5;
  pow_series_par(gp, glen, g, threads);
  memcpy(layer, code, n0 * 16);
  uint64_t n = n0;
  uint32_t t = 0;
  merkle_pairs_par((const uint8_t*)layer, log_code, tree, threads);
  memcpy(roots + 32 * t, tree + 32 * (n - 2), 32);
  sha_update(&tr, roots + 32 * t, 32);
  t++;
  int rc = 0;
  for (uint32_t k = 0; k + 1 < log_code; k++) {
    uint8_t rnd[32];
    sha_final(&tr, rnd);
    u128 r = ld(rnd);
    if (r >= MOD) r -= MOD;
    const uint64_t half = n / 2;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long ii = 0; ii < (long long)half; ii++) {
      const uint64_t i = (uint64_t)ii;
      const u128 a = layer[i], b = layer[i + half];
      const u128 tw = i == 0 ? 1 : gp[glen - i * (1ull << k)];
      const u128 odd = fmul(fsub(a, b), tw);
      next[i] = fmul(fadd(fadd(a, b), fmul(r, odd)), inv2);
    }
    memcpy(layer, next, half * 16);
    n = half;
    if (half == 2) {
      if (layer[0] != layer[1]) rc = 6;
      st(last, layer[0]);
      sha_update(&tr, last, 16);
      break;
    }
    merkle_pairs_par((const uint8_t*)layer, (uint32_t)__builtin_ctzll(n), tree, threads);
    memcpy(roots + 32 * t, tree + 32 * (n - 2), 32);
    sha_update(&tr, roots + 32 * t, 32);
    t++;
  }
  if (last_random) sha_final(&tr, last_random);
  free(layer);
  free(next);
  free(tree);
  free(gp);
  return rc;
}

void orc_eq_table_par(const uint8_t* pts, uint32_t n, uint8_t* out, int threads) {
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long ii = 0; ii < (long long)(1ull << n); ii++) {
    const uint64_t idx = (uint64_t)ii;
    u128 acc = 1;
    for (uint32_t i = 0; i < n; i++) {
      const u128 p = ld(pts + 16 * (n - 1 - i));
      acc = fmul(acc, ((idx >> i) & 1) ? p : fsub(1, p));
    }
    st(out + 16 * idx, acc);
  }
}

void orc_partial_sums_par(const uint8_t* m, const uint8_t* d, uint32_t log_h, uint8_t out[32],
                          int threads) {
  const uint64_t off = (1ull << log_h) / 2;
  u128 s1 = 0, s2 = 0;
  const u128 r = 2, s = fsub(1, r);
#pragma omp parallel num_threads(threads)
  {
    u128 a1 = 0, a2 = 0;
#pragma omp for schedule(static)
    for (long long ii = 0; ii < (long long)off; ii++) {
      const uint64_t i = (uint64_t)ii;
      a1 = fadd(a1, fmul(ld(m + 16 * (i + off)), ld(d + 16 * (i + off))));
      const u128 dd = fadd(fmul(s, ld(d + 16 * i)), fmul(r, ld(d + 16 * (i + off))));
      const u128 mm = fadd(fmul(s, ld(m + 16 * i)), fmul(r, ld(m + 16 * (i + off))));
      a2 = fadd(a2, fmul(mm, dd));
    }
#pragma omp critical
    {
      s1 = fadd(s1, a1);
      s2 = fadd(s2, a2);
    }
  }
  st(out, s1);
  st(out + 16, s2);
}

void orc_fold_par(uint8_t* m, uint8_t* d, uint32_t log_h, const uint8_t rb[16], int threads) {
  const uint64_t off = (1ull << log_h) / 2;
  const u128 r = ld(rb), s = fsub(1, r);
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long ii = 0; ii < (long long)off; ii++) {
    const uint64_t i = (uint64_t)ii;
    st(d + 16 * i, fadd(fmul(s, ld(d + 16 * i)), fmul(r, ld(d + 16 * (i + off)))));
    st(m + 16 * i, fadd(fmul(s, ld(m + 16 * i)), fmul(r, ld(m + 16 * (i + off)))));
  }
}

/* sum_i m[i] d[i] (the claimed sum of the PCS sumcheck, polynomials.rs:165-187
 * as an eq-table dot product) */
void orc_dot_par(const uint8_t* m, const uint8_t* d, uint32_t log_n, uint8_t out[16], int threads) {
  u128 tot = 0;
#pragma omp parallel num_threads(threads)
  {
    u128 acc = 0;
#pragma omp for schedule(static)
    for (long long ii = 0; ii < (long long)(1ull << log_n); ii++)
      acc = fadd(acc, fmul(ld(m + 16 * (uint64_t)ii), ld(d + 16 * (uint64_t)ii)));
#pragma omp critical
    tot = fadd(tot, acc);
  }
  st(out, tot);
}

/* ============================================ whole PCS / batched PCS prove */
/* PCSProof::prove (src/fri/multilinear_pcs.rs:90-136, PCSProverData::fold
 * :43-76) and BatchedPCSProof::prove (src/fri/batched_pcs.rs:127-180,
 * BatchedPCSProverData::{init,fold} :36-125), restated end to end in C so the
 * production-shape GPU prove (n = 19..24 variables; batched (10, 20)) can be
 * compared byte for byte: every round polynomial, the batch root, every fold
 * root, the last element, the final transcript digest and all 128 query
 * records.  The reference order is kept: to_coefficient -> bit reversal ->
 * reed_solomon; FriProverData::init; per round compute_sumcheck_polynomial
 * (sumcheck.rs:174-202: partial_sum at 1 and 2, Lagrange interpolation on
 * 0,1,2, absorb the two nonzero coefficients, next_challenge, fold) then
 * fold_step (fri/mod.rs:79-134) with the same r; queries as fri/mod.rs:268-277
 * and open_query_at :154-175.  OpenMP only splits independent loops (leaves,
 * pairs, table entries); every field value is exact, so the result does not
 * depend on the thread count. */

typedef struct {
  uint64_t len;  /* values in the layer; pairs (i, i + len/2) */
  u128* vals;
  uint8_t* tree; /* (len - 1) * 32: len/2 leaf digests, then each level */
} orc_layer;

static u128 tr_challenge(const sha_t* tr) { /* transcript.rs next_challenge */
  uint8_t rnd[32];
  sha_final(tr, rnd);
  u128 r = ld(rnd);
  return r >= MOD ? r - MOD : r;
}

static void commit_layer(orc_layer* ly, int threads) { /* commit_rs_code, fri/mod.rs:45-55 */
  ly->tree = (uint8_t*)malloc((ly->len - 1) * 32);
  merkle_pairs_par((const uint8_t*)ly->vals, (uint32_t)__builtin_ctzll(ly->len), ly->tree, threads);
}
static const uint8_t* layer_root(const orc_layer* ly) { return ly->tree + 32 * (ly->len - 2); }

/* Merkle::open (merkle_tree/mod.rs:31-58) of the pair at idx: value bytes,
 * then the sibling of every level below the root.  Returns bytes written. */
static uint64_t open_layer(const orc_layer* ly, uint64_t idx, uint8_t* out) {
  const uint64_t L = ly->len / 2;
  st(out, ly->vals[idx]);
  st(out + 16, ly->vals[idx + L]);
  uint64_t w = 32, off = 0, cnt = L, cur = idx;
  while (cnt > 1) {
    memcpy(out + w, ly->tree + 32 * (off + (cur ^ 1)), 32);
    w += 32;
    off += cnt;
    cnt /= 2;
    cur /= 2;
  }
  return w;
}

/* the fold loop of fold_step (fri/mod.rs:89-114): next[i] =
 * ((a + b) + r (a - b) gen_pows[len - i 2^k]) / 2, i = 0 with twiddle 1 */
static void fold_layer_par(const u128* src, uint64_t n, const u128* gp, uint64_t glen, uint32_t k, u128 r,
                           u128* dst, int threads) {
  const uint64_t half = n / 2;
  const u128 inv2 = finv(2);
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long ii = 0; ii < (long long)half; ii++) {
    const uint64_t i = (uint64_t)ii;
    const u128 a = src[i], b = src[i + half];
    const u128 tw = i == 0 ? 1 : gp[glen - i * (1ull << k)];
    dst[i] = fmul(fadd(fadd(a, b), fmul(r, fmul(fsub(a, b), tw))), inv2);
  }
}

/* Horner fingerprint (batched_fri.rs:30-38): ((c_0 r + c_1) r + ...) + c_{m-1} */
static u128 fingerprint_col(u128 r, const u128* base, uint64_t stride, uint32_t m, uint64_t i) {
  u128 acc = 0;
  for (uint32_t j = 0; j < m; j++) acc = fadd(fmul(acc, r), base[(uint64_t)j * stride + i]);
  return acc;
}

/* PolynomialEvals::interpolate (polynomials.rs:51-87) on x = 0, 1, 2 */
static void interpolate3(const u128 e[3], u128 c[3]) {
  c[0] = c[1] = c[2] = 0;
  for (int j = 0; j < 3; j++) {
    u128 lj[3] = {1, 0, 0}, denom = 1;
    int deg = 0;
    for (int m = 0; m < 3; m++) {
      if (m == j) continue;
      u128 nl[3] = {0, 0, 0};
      for (int i = 0; i <= deg; i++) {
        nl[i] = fsub(nl[i], fmul(lj[i], (u128)m));
        nl[i + 1] = fadd(nl[i + 1], lj[i]);
      }
      deg++;
      memcpy(lj, nl, sizeof nl);
      denom = fmul(denom, j >= m ? (u128)(j - m) : fsub(0, (u128)(m - j)));
    }
    const u128 sc = fmul(e[j], finv(denom));
    for (int i = 0; i < 3; i++) c[i] = fadd(c[i], fmul(sc, lj[i]));
  }
}

/* one compute_sumcheck_polynomial (sumcheck.rs:174-202) on (mt, dt) of 2^lh
 * entries with composition x[0]; writes c1 || c2, absorbs them, returns r and
 * folds the tables in place (sumcheck.rs:234-247). */
static u128 sumcheck_round(u128* mt, u128* dt, uint32_t lh, u128* prev, sha_t* tr, uint8_t out[32],
                           int threads) {
  const uint64_t off = (1ull << lh) / 2;
  u128 s1 = 0, s2 = 0;
  const u128 two = 2, mone = fsub(1, two);
#pragma omp parallel num_threads(threads)
  {
    u128 a1 = 0, a2 = 0;
#pragma omp for schedule(static)
    for (long long ii = 0; ii < (long long)off; ii++) {
      const uint64_t i = (uint64_t)ii;
      a1 = fadd(a1, fmul(mt[i + off], dt[i + off]));
      const u128 dd = fadd(fmul(mone, dt[i]), fmul(two, dt[i + off]));
      const u128 mm = fadd(fmul(mone, mt[i]), fmul(two, mt[i + off]));
      a2 = fadd(a2, fmul(mm, dd));
    }
#pragma omp critical
    {
      s1 = fadd(s1, a1);
      s2 = fadd(s2, a2);
    }
  }
  const u128 e[3] = {fsub(*prev, s1), s1, s2};
  u128 c[3];
  interpolate3(e, c);
  st(out, c[1]);
  st(out + 16, c[2]);
  sha_update(tr, out, 32);
  const u128 r = tr_challenge(tr);
  *prev = fadd(c[0], fmul(r, fadd(c[1], fmul(r, c[2]))));
  const u128 s = fsub(1, r);
#pragma omp parallel for num_threads(threads) schedule(static)
  for (long long ii = 0; ii < (long long)off; ii++) {
    const uint64_t i = (uint64_t)ii;
    dt[i] = fadd(fmul(s, dt[i]), fmul(r, dt[i + off]));
    mt[i] = fadd(fmul(s, mt[i]), fmul(r, mt[i + off]));
  }
  return r;
}

/* Bytes of one query record in the flat layout written below (the layout
 * libmlhip's query staging uses): unbatched, per tree t < n: pair (32 B) +
 * (n - t) siblings; batched, the column (m x 32 B) + n batch-path siblings,
 * then per inner tree t < n - 1: pair + (n - 1 - t) siblings. */
uint64_t orc_pcs_query_bytes(uint32_t m, uint32_t n, int batched) {
  uint64_t b = 0;
  if (!batched) {
    for (uint32_t t = 0; t < n; t++) b += 32ull * (1 + n - t);
    return b;
  }
  b = 32ull * m + 32ull * n;
  for (uint32_t t = 0; t + 1 < n; t++) b += 32ull * (n - t);
  return b;
}

/* evals: m x 2^n (poly-major); points: n; outputs: m claims (unbatched: m = 1,
 * the claimed evaluation).  prefix bytes are absorbed into the fresh
 * transcript first.  Outputs: polys n x 32 (c1 || c2), batch_root 32
 * (batched only), roots (n - batched) x 32, last 16, last_random 32, qidx 128,
 * qrec 128 x orc_pcs_query_bytes.  Returns 0, 2 (bad shape), 5 (alloc) or 6
 * (the last layer is not constant: "not an RS code"). */
int orc_pcs_prove_par(const uint8_t* evals, uint32_t m, uint32_t n, const uint8_t* points,
                      const uint8_t* outputs, int batched, const uint8_t* prefix, uint64_t prefix_len,
                      uint8_t* polys, uint8_t* batch_root, uint8_t* roots, uint8_t last[16],
                      uint8_t last_random[32], uint64_t* qidx, uint8_t* qrec, int threads) {
  if (n < 1 || m < 1 || (!batched && m != 1) || n > 30) return 2;
  const uint64_t H = 1ull << n, N0 = 2 * H; /* evaluations, code length */
  const uint32_t log_dom = n + 1;            /* + LOG_BLOWUP */
  sha_t tr;
  sha_init(&tr);
  if (prefix_len) sha_update(&tr, prefix, prefix_len);
  /* gen_pows = pow_2_generator_powers(log_domain) (multilinear_pcs.rs:97-99) */
  u128* gp = (u128*)malloc(N0 * sizeof(u128));
  u128* codes = (u128*)malloc((uint64_t)m * N0 * sizeof(u128));
  orc_layer* lay = (orc_layer*)calloc(n + 1, sizeof(orc_layer));
  u128* mt = (u128*)malloc(H * sizeof(u128));
  u128* dt = (u128*)malloc(H * sizeof(u128));
  if (!gp || !codes || !lay || !mt || !dt) return 5;
  const u128 g = fpow(3, (MOD - 1) >> log_dom);
  pow_series_par(gp, N0, g, threads);
  uint8_t gb[16];
  st(gb, gp[1]);
  /* per polynomial: to_coefficient, bit_reverse_permutation, reed_solomon */
  for (uint32_t j = 0; j < m; j++) {
    u128* c = codes + (uint64_t)j * N0;
    memcpy(c, evals + 16 * (uint64_t)j * H, H * 16);
    for (uint32_t i = 0; i < n; i++) { /* polynomials.rs:150-163 */
      const uint64_t msk = 1ull << i;
#pragma omp parallel for num_threads(threads) schedule(static)
      for (long long jj = 0; jj < (long long)H; jj++)
        if ((uint64_t)jj & msk) c[jj] = fsub(c[jj], c[(uint64_t)jj ^ msk]);
    }
    bit_reverse_permutation(c, H);
    memset(c + H, 0, H * 16);
    orc_ntt_par((const uint8_t*)c, (uint8_t*)c, log_dom, gb, 0, threads);
  }
  /* claim absorb + first commitment */
  u128 fr = 0, prev;
  uint8_t* batch_tree = NULL;
  if (batched) {
    for (uint32_t i = 0; i < n; i++) sha_update(&tr, points + 16 * i, 16);
    for (uint32_t j = 0; j < m; j++) sha_update(&tr, outputs + 16 * j, 16);
    /* BatchedFriProverData::init (batched_fri.rs:41-98): Merkle::batch_commit
     * of the per-code RS pairs, leaf i = SHA256(pair_0[i] || pair_1[i] || ..) */
    batch_tree = (uint8_t*)malloc((2 * H - 1) * 32);
    if (!batch_tree) return 5;
#pragma omp parallel num_threads(threads)
    {
      uint8_t* buf = (uint8_t*)malloc(32ull * m);
#pragma omp for schedule(static)
      for (long long ii = 0; ii < (long long)H; ii++) {
        for (uint32_t j = 0; j < m; j++) {
          st(buf + 32ull * j, codes[(uint64_t)j * N0 + (uint64_t)ii]);
          st(buf + 32ull * j + 16, codes[(uint64_t)j * N0 + (uint64_t)ii + H]);
        }
        orc_sha256(buf, 32ull * m, batch_tree + 32 * (uint64_t)ii);
      }
      free(buf);
    }
    uint64_t off = 0, cnt = H;
    while (cnt > 1) {
#pragma omp parallel for num_threads(threads) schedule(static) if (cnt > 4096)
      for (long long jn = 0; jn < (long long)(cnt / 2); jn++)
        orc_sha256(batch_tree + 32 * (off + 2 * (uint64_t)jn), 64, batch_tree + 32 * (off + cnt + (uint64_t)jn));
      off += cnt;
      cnt /= 2;
    }
    memcpy(batch_root, batch_tree + 32 * (2 * H - 2), 32);
    sha_update(&tr, batch_root, 32);
    fr = tr_challenge(&tr);
    uint8_t fb[16];
    st(fb, fr);
    sha_update(&tr, fb, 16);
    /* fingerprinted evaluations -> the sumcheck matrix (batched_pcs.rs:54-64) */
    u128* ev = (u128*)malloc((uint64_t)m * H * sizeof(u128));
    if (!ev) return 5;
    memcpy(ev, evals, (uint64_t)m * H * 16);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long ii = 0; ii < (long long)H; ii++) mt[ii] = fingerprint_col(fr, ev, H, m, (uint64_t)ii);
    free(ev);
    u128* outs = (u128*)malloc(m * sizeof(u128));
    for (uint32_t j = 0; j < m; j++) outs[j] = ld(outputs + 16 * j);
    prev = fingerprint_col(fr, outs, 1, m, 0);
    free(outs);
  } else {
    /* FriProverData::init (fri/mod.rs:58-76) */
    lay[0].len = N0;
    lay[0].vals = codes;
    commit_layer(&lay[0], threads);
    sha_update(&tr, layer_root(&lay[0]), 32);
    memcpy(mt, evals, H * 16);
    prev = ld(outputs);
  }
  /* build_tables_for_pcs (sumcheck.rs:128-145): delta = eq(points), big endian */
  dt[0] = 1;
  for (uint32_t i = n; i-- > 0;) {
    const uint64_t cur = 1ull << (n - 1 - i);
    const u128 p = ld(points + 16 * i), q = fsub(1, p);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (long long jj = 0; jj < (long long)cur; jj++) {
      dt[(uint64_t)jj + cur] = fmul(dt[jj], p);
      dt[jj] = fmul(dt[jj], q);
    }
  }
  /* rounds: compute_sumcheck_polynomial, then fold_step with the same r */
  uint32_t nl = batched ? 0 : 1; /* committed FRI layers */
  int rc = 0;
  u128 last_el = 0;
  for (uint32_t k = 0; k < n; k++) {
    const u128 r = sumcheck_round(mt, dt, n - k, &prev, &tr, polys + 32 * k, threads);
    const u128* src;
    uint64_t len;
    u128* fpv = NULL;
    if (batched && k == 0) { /* batched_fold_step (batched_fri.rs:100-176) */
      fpv = (u128*)malloc(N0 * sizeof(u128));
      if (!fpv) return 5;
#pragma omp parallel for num_threads(threads) schedule(static)
      for (long long ii = 0; ii < (long long)N0; ii++) fpv[ii] = fingerprint_col(fr, codes, N0, m, (uint64_t)ii);
      src = fpv;
      len = N0;
    } else {
      src = lay[nl - 1].vals;
      len = lay[nl - 1].len;
    }
    if (len <= 2) break;
    u128* nxt = (u128*)malloc((len / 2) * sizeof(u128));
    if (!nxt) return 5;
    fold_layer_par(src, len, gp, N0, k, r, nxt, threads);
    free(fpv);
    if (len / 2 == 2) {
      if (nxt[0] != nxt[1]) rc = 6;
      last_el = nxt[0];
      st(last, last_el);
      sha_update(&tr, last, 16);
      free(nxt);
      break;
    }
    lay[nl].len = len / 2;
    lay[nl].vals = nxt;
    commit_layer(&lay[nl], threads);
    sha_update(&tr, layer_root(&lay[nl]), 32);
    nl++;
  }
  for (uint32_t t = 0; t < nl; t++) memcpy(roots + 32 * t, layer_root(&lay[t]), 32);
  /* queries (multilinear_pcs.rs:113-121 / batched_pcs.rs:160-168) */
  const uint64_t qb = orc_pcs_query_bytes(m, n, batched);
  for (int q = 0; q < 128; q++) {
    uint8_t rnd[32];
    sha_final(&tr, rnd);
    uint64_t r64;
    memcpy(&r64, rnd, 8);
    const uint64_t idx = r64 % (N0 / 2);
    qidx[q] = idx;
    uint8_t* o = qrec + qb * (uint64_t)q;
    uint64_t cur = idx;
    if (batched) { /* batched open_query_at (batched_fri.rs:207-224) */
      for (uint32_t j = 0; j < m; j++) {
        st(o, codes[(uint64_t)j * N0 + idx]);
        st(o + 16, codes[(uint64_t)j * N0 + idx + H]);
        o += 32;
      }
      uint64_t off = 0, cnt = H, c2 = idx;
      while (cnt > 1) {
        memcpy(o, batch_tree + 32 * (off + (c2 ^ 1)), 32);
        o += 32;
        off += cnt;
        cnt /= 2;
        c2 /= 2;
      }
      cur = idx % (H / 2);
    }
    for (uint32_t t = 0; t < nl; t++) { /* open_query_at (fri/mod.rs:154-175) */
      o += open_layer(&lay[t], cur, o);
      cur %= lay[t].len / 4 ? lay[t].len / 4 : 1;
    }
    sha_update(&tr, (const uint8_t*)&idx, 8);
  }
  sha_final(&tr, last_random);
  for (uint32_t t = batched ? 0 : 1; t < nl; t++) free(lay[t].vals);
  for (uint32_t t = 0; t < nl; t++) free(lay[t].tree);
  free(lay);
  free(batch_tree);
  free(codes);
  free(gp);
  free(mt);
  free(dt);
  return rc;
}
