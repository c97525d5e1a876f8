/*
 * mlhip.h -- C ABI of the MI355X (gfx950) proving backend for the hot path of
 * fr34za/multilinear (reference @ 2025-06-20): radix-2 NTT, Reed-Solomon LDE,
 * SHA-256 Merkle level hashing, FRI layer folding, and MLE/sumcheck round
 * sums over the field.rs prime M = 2^128 - 45*2^40 + 1.
 *
 * Conventions (identical to the reference's in-memory forms):
 *   - a field element is 16 bytes: the canonical u128 (value < M), little
 *     endian -- Field128::as_ref (src/field.rs:33-38);
 *   - a digest is the 32 SHA-256 output bytes (HashDigest, merkle_tree/mod.rs:5);
 *   - a Merkle tree of L = 2^l leaves is one buffer of 2L-1 digests in level
 *     order (leaves first, root last) -- Merkle::layers flattened
 *     (merkle_tree/mod.rs:7-11);
 *   - "dev" pointers are device (HBM) pointers on the context's device, e.g.
 *     from mlh_malloc or any HIP allocator; "host" pointers are host memory.
 *   - All work is enqueued on the context's HIP stream; functions that return
 *     host results (roots, sums, proofs) synchronise that stream.
 *
 * Errors: the reference prover panics (assert!) on non-power-of-two sizes,
 * bad lengths and the "not an RS code" check; here every entry point returns
 * an mlh_status and mlh_last_error() gives the message.  Nothing falls back
 * to a CPU implementation: without a usable gfx950 device every compute call
 * returns MLH_ERR_HIP.
 */
#ifndef MLHIP_H
#define MLHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mlh_status {
  MLH_OK = 0,
  MLH_ERR_INVALID = 1,       /* bad argument (null pointer, size out of range)   */
  MLH_ERR_NOT_POW2 = 2,      /* "must be a power of two" asserts                   */
  MLH_ERR_BAD_GENERATOR = 3, /* generator not canonical, or (FRI / sharded entry
                                points) not of order exactly 2^log_n              */
  MLH_ERR_HIP = 4,           /* HIP runtime error / no device                      */
  MLH_ERR_OOM = 5,           /* device allocation failed                           */
  MLH_ERR_NOT_RS_CODE = 6,   /* fri/mod.rs:119-122 "not an RS code"                */
  MLH_ERR_VERIFY = 7,        /* verifier rejected (Merkle: IncompatibleHash)       */
  MLH_ERR_VERIFY_INDEX = 8,  /* Merkle path directions != index (IncompatibleIndex) */
  MLH_ERR_COMM = 9,          /* a collective of the multi-GPU transport failed      */
  MLH_ERR_DEVICE = 10        /* device-side failure inside a prove: a cooperative
                                kernel's wait timed out, or a challenge the device
                                drew differs from the host transcript replay; the
                                outputs of that call are invalid and the caller's
                                transcript is left as it was at the call's entry */
} mlh_status;

typedef struct mlh_ctx mlh_ctx;               /* device + stream + twiddle caches */
typedef struct mlh_transcript mlh_transcript; /* transcript.rs Transcript         */
typedef struct mlh_fri_prover mlh_fri_prover; /* fri/mod.rs FriProverData         */

#define MLH_LOG_BLOWUP 1   /* fri/mod.rs:16 */
#define MLH_NUM_QUERIES 128 /* fri/mod.rs:17 */

/* ---- context and memory ------------------------------------------------- */
const char* mlh_version(void);
mlh_status mlh_context_create(int device, void* hip_stream, mlh_ctx** out);
void mlh_context_destroy(mlh_ctx* ctx);
/* Twiddle / fold tables are cached per context (built on the first use of a
 * size and generator) in a bounded LRU cache: default limit 1 GiB; tables the
 * running operation uses are never evicted, so the cache may exceed a very
 * small limit by that operation's tables.  limit 0 frees every table not in
 * use at the next opportunity.  The largest: an FRI prove of a codeword of
 * 2^L <= 2^25 elements caches every fold layer's twiddles in one table of
 * 2^L - 1 entries (512 MiB at 2^25); above 2^25 the folds form them from two
 * 4096-entry tables instead.  A 2^23 or 2^24 NTT's first pass adds a 64 x 2^16
 * progression table and its 2^16-entry step table (68 MiB at 2^24). */
mlh_status mlh_set_table_cache_limit(mlh_ctx* ctx, uint64_t bytes);
uint64_t mlh_table_cache_bytes(const mlh_ctx* ctx);
/* Test/tuning hook: force the NTT radix plan of this context (count digits
 * 4..9; a plan applies to the transforms whose log size equals its digit sum;
 * count = 0 restores the default plan). */
mlh_status mlh_set_ntt_plan(mlh_ctx* ctx, const uint32_t* logr, uint32_t count);
/* Test hook: the cooperative sumcheck kernels' wait limit, in s_sleep(1)
 * periods (0 restores the default 2^22).  A wait that exceeds it abandons the
 * kernel's rounds and the prove returns MLH_ERR_DEVICE. */
mlh_status mlh_set_coop_spin_limit(mlh_ctx* ctx, uint32_t sleeps);
/* Test hook: the PCS and batched PCS provers compute their sumcheck rounds
 * off the transcript chain for n_vars <= max_vars (default and cap 24) and
 * with one cooperative launch per round above it; both give the same proof. */
mlh_status mlh_set_pcs_fused_max(mlh_ctx* ctx, uint32_t max_vars);
mlh_status mlh_set_stream(mlh_ctx* ctx, void* hip_stream);
mlh_status mlh_synchronize(mlh_ctx* ctx);
/* The message of ctx's last failure; with ctx == NULL, why this thread's last
 * mlh_context_create failed. */
const char* mlh_last_error(const mlh_ctx* ctx);
mlh_status mlh_malloc(mlh_ctx* ctx, size_t bytes, void** dev);
mlh_status mlh_free(mlh_ctx* ctx, void* dev);
mlh_status mlh_memcpy_h2d(mlh_ctx* ctx, void* dev, const void* host, size_t bytes);
mlh_status mlh_memcpy_d2h(mlh_ctx* ctx, void* host, const void* dev, size_t bytes);
mlh_status mlh_memcpy_d2d(mlh_ctx* ctx, void* dst, const void* src, size_t bytes);

/* ---- field helpers (host) ------------------------------------------------ */
/* NttField::pow_2_generator (src/ntt/mod.rs:42-54): 3^((M-1)/2^log_size). */
mlh_status mlh_pow_2_generator(uint32_t log_size, uint8_t gen_out[16]);
/* NttField::pow_2_generator_powers (src/ntt/mod.rs:18-28): out[i] = g^i,
 * i < 2^log_size, written to dev (no serial chain on the device). */
mlh_status mlh_pow_2_generator_powers(mlh_ctx* ctx, uint32_t log_size, void* dev_out);

/* Elementwise Field128 ops on device vectors of n elements (src/field.rs:66-111:
 * Add, Sub, Mul, Neg).  Inputs canonical; out may alias an input. */
mlh_status mlh_field_add(mlh_ctx* ctx, const void* dev_a, const void* dev_b, void* dev_out, uint64_t n);
mlh_status mlh_field_sub(mlh_ctx* ctx, const void* dev_a, const void* dev_b, void* dev_out, uint64_t n);
mlh_status mlh_field_mul(mlh_ctx* ctx, const void* dev_a, const void* dev_b, void* dev_out, uint64_t n);
mlh_status mlh_field_neg(mlh_ctx* ctx, const void* dev_a, void* dev_out, uint64_t n);
/* out[i] = a[i] * c (scalar Mul, field.rs:98-106); c canonical LE16. */
mlh_status mlh_field_scale(mlh_ctx* ctx, const void* dev_a, const uint8_t c[16], void* dev_out,
                           uint64_t n);

/* ---- NTT (src/ntt/mod.rs) ------------------------------------------------ */
/* Polynomial::ntt (ntt/mod.rs:69-110): evals[i] = sum_j coeffs[j] gen^(ij),
 * natural order in and out, when gen has order exactly 2^log_n (the fast
 * passes).  Any other canonical gen (0 included) gets the reference's own
 * bit-reverse + radix-2 network output -- well defined but not a DFT -- from a
 * stage-by-stage path (log_n + 1 - 11 launches; a correctness path, not tuned).
 * In-place (dev_in == dev_out) is allowed. */
mlh_status mlh_ntt(mlh_ctx* ctx, const void* dev_coeffs, void* dev_evals, uint32_t log_n,
                   const uint8_t gen[16]);
/* LagrangePolynomial::intt (ntt/mod.rs:132-173): gen is the forward
 * generator (LagrangePolynomial::gen); uses gen^-1 (0 for gen = 0, as
 * winter-math's inverse) and scales by 1/n.  Generators as mlh_ntt. */
mlh_status mlh_intt(mlh_ctx* ctx, const void* dev_evals, void* dev_coeffs, uint32_t log_n,
                    const uint8_t gen[16]);
/* bit_reverse_permutation (ntt/mod.rs:113-123), out of place (in != out);
 * log_n >= 1 (n = 1 panics in the reference: MLH_ERR_NOT_POW2). */
mlh_status mlh_bit_reverse_permutation(mlh_ctx* ctx, const void* dev_in, void* dev_out,
                                       uint32_t log_n);
/* Vec -> Vec convenience (host buffers, includes PCIe copies). */
mlh_status mlh_ntt_host(mlh_ctx* ctx, const uint8_t* host_in, uint8_t* host_out, uint32_t log_n,
                        const uint8_t gen[16], int inverse);

/* ---- Reed-Solomon, Merkle, FRI (src/fri, src/merkle_tree) -------------------- */
/* reed_solomon (fri/mod.rs:19-28): zero-pad 2^log_n coeffs to 2^(log_n+1) and
 * NTT with gen (order 2^(log_n+1); any other canonical gen as mlh_ntt).
 * dev_code holds 2^(log_n+1) elements. */
mlh_status mlh_reed_solomon(mlh_ctx* ctx, const void* dev_coeffs, uint32_t log_n,
                            const uint8_t gen[16], void* dev_code);
/* reed_solomon(bit_reverse_permutation(coeffs)) in one transform: the commit
 * step of multilinear_pcs.rs:104-107 / batched_pcs.rs:146-147 with the
 * permutation folded into the first pass's loads (out of place). */
mlh_status mlh_reed_solomon_brev(mlh_ctx* ctx, const void* dev_coeffs, uint32_t log_n,
                                 const uint8_t gen[16], void* dev_code);
/* Bytes of a flattened tree with `leaves` leaves: (2*leaves - 1) * 32. */
uint64_t mlh_merkle_layers_bytes(uint64_t leaves);
/* commit_rs_code (fri/mod.rs:45-55) + Merkle::commit (merkle_tree/mod.rs:65-85):
 * leaf i = SHA256(LE16(code[i]) ‖ LE16(code[i + n/2])), n = 2^log_code. */
mlh_status mlh_merkle_commit_pairs(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                   void* dev_layers, uint8_t root_out[32]);
/* Merkle::commit over `count` (power of two) items of item_len bytes each. */
mlh_status mlh_merkle_commit(mlh_ctx* ctx, const void* dev_items, uint64_t item_len,
                             uint64_t count, void* dev_layers, uint8_t root_out[32]);
/* Merkle::batch_commit (merkle_tree/mod.rs:92-131): m batches of `count`
 * items, batch j at dev_items + j*count*item_len; leaf i hashes the m items i. */
mlh_status mlh_merkle_batch_commit(mlh_ctx* ctx, const void* dev_items, uint64_t item_len,
                                   uint32_t m, uint64_t count, void* dev_layers,
                                   uint8_t root_out[32]);
/* The fold loop of FriProverData::fold_step (fri/mod.rs:89-114): layer of
 * 2^log_layer values (pairs i, i + n/2) -> 2^(log_layer-1) values, fold index
 * k, original domain 2^log_domain (twiddle g^(-i 2^k)). */
mlh_status mlh_fri_fold(mlh_ctx* ctx, const void* dev_layer, uint32_t log_layer, uint32_t k,
                        uint32_t log_domain, const uint8_t r[16], void* dev_next);

/* FriProverData (fri/mod.rs:10-175), device resident.
 * gen_pows: the reference's FriProverData::{init,fold} and FriProof::prove
 * take the table gen_pows and fold with twiddle gen_pows[gen_pows.len() - i 2^k]
 * (fri/mod.rs:106-110).  The plain entry points assume the canonical table of
 * the code's own length (pow_2_generator_powers(log_code), what every reference
 * caller passes); the _gp variants take the table as (gen_pows[1],
 * log2(gen_pows.len())) for any geometric table of a generator of order exactly
 * gen_pows.len() (MLH_ERR_BAD_GENERATOR otherwise; MLH_ERR_INVALID when the
 * table is shorter than half the code, where the reference's index underflows). */
/* The shim from the reference's gen_pows: &[F] (fri/mod.rs:79, :136, :261) to
 * the _gp arguments: returns (g = gen_pows[1], log2(len)) after checking, on
 * the host, that len is a power of two >= 2, g has order exactly len, and the
 * table agrees with 1, g, g^2, ... at every index < min(len, 4096), at every
 * 2^j, at len/2 (= -1), at len-1 (= g^-1) and at 16 pseudo-random indices
 * (MLH_ERR_INVALID otherwise).  That is a spot check: a table altered only
 * elsewhere passes it, and the library would then fold with the true powers
 * where the reference folds with the altered entry (fri/mod.rs:110).  The full
 * check is mlh_gen_pows_verify. */
mlh_status mlh_gen_pows_params(const uint8_t* gen_pows, uint64_t len, uint8_t gen_out[16],
                               uint32_t* log_len_out);
/* Full check of a host gen_pows table: every entry against g^i on the device
 * (one pass of the table over PCIe, ~16 B per entry, plus one comparison
 * kernel), after mlh_gen_pows_params' checks.  MLH_OK iff the table IS the
 * power series of gen_pows[1] (of order len); otherwise MLH_ERR_INVALID with
 * the first differing index in mlh_last_error().  gen_out / log_len_out as
 * mlh_gen_pows_params (either may be null).  A caller that reuses one table for
 * many proofs verifies it once. */
mlh_status mlh_gen_pows_verify(mlh_ctx* ctx, const uint8_t* gen_pows, uint64_t len,
                               uint8_t gen_out[16], uint32_t* log_len_out);
mlh_status mlh_fri_prover_init(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                               mlh_transcript* tr, mlh_fri_prover** out); /* :58-76  */
mlh_status mlh_fri_prover_init_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                  const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                  mlh_transcript* tr, mlh_fri_prover** out);
/* fold_step(&mut self, gen_pows, k, r, transcript) (fri/mod.rs:79-134).  The
 * plain form folds with the table the prover was created with (init: the
 * code's canonical table); _gp takes the caller's table for this step, as the
 * reference does at every call (multilinear_pcs.rs:72, batched_pcs.rs:121,
 * batched_fri.rs:200, fri/mod.rs:141): twiddle gen_pows[len - i 2^k] =
 * gen_pows_1^(-(i 2^k) mod len) for a table of 2^log_gen_pows powers of a
 * generator of that exact order (MLH_ERR_BAD_GENERATOR otherwise).  Any k is
 * accepted while (n/2 - 1) 2^k <= len (beyond it the reference's index
 * underflows: MLH_ERR_INVALID).  Like the reference, a step after the last
 * element folds the last tree again and re-absorbs the element. */
mlh_status mlh_fri_prover_fold_step(mlh_ctx* ctx, mlh_fri_prover* p, uint32_t k,
                                    const uint8_t r[16], mlh_transcript* tr); /* :79-134 */
mlh_status mlh_fri_prover_fold_step_gp(mlh_ctx* ctx, mlh_fri_prover* p, const uint8_t gen_pows_1[16],
                                       uint32_t log_gen_pows, uint32_t k, const uint8_t r[16],
                                       mlh_transcript* tr);
mlh_status mlh_fri_prover_fold(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                               mlh_transcript* tr, mlh_fri_prover** out); /* :136-145 */
mlh_status mlh_fri_prover_fold_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                  const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                  mlh_transcript* tr, mlh_fri_prover** out);
uint32_t mlh_fri_prover_num_trees(const mlh_fri_prover* p);
mlh_status mlh_fri_prover_roots(const mlh_fri_prover* p, uint8_t* roots_out /* [T][32] */);
/* last_element (fri/mod.rs:13); MLH_ERR_INVALID while still None. */
mlh_status mlh_fri_prover_last_element(const mlh_fri_prover* p, uint8_t out[16]);
/* open_query_at (fri/mod.rs:154-175) -> one query record (layout below). */
mlh_status mlh_fri_prover_open_query(mlh_ctx* ctx, const mlh_fri_prover* p, uint64_t index,
                                     uint8_t* out);
void mlh_fri_prover_destroy(mlh_fri_prover* p);

/* FriProof (fri/mod.rs:239-249) as caller-allocated flat buffers.
 * Query record for a code of 2^L elements: for tree t = 0..L-2: the opened
 * ReedSolomonPair (32 B) then its L-1-t sibling digests leaf-to-root (32 B
 * each); the Direction of level i is Right iff bit i of the opened index is 0
 * (merkle_tree/mod.rs:43-47), so it is not stored. */
typedef struct mlh_fri_proof {
  uint32_t log_code;    /* L = log2(code length)                    */
  uint32_t num_trees;   /* commitments: L - MLH_LOG_BLOWUP          */
  uint32_t num_queries; /* MLH_NUM_QUERIES                          */
  uint8_t* commitments; /* [num_trees][32]                         */
  uint8_t last_elem[16];
  uint8_t last_random[32];
  uint64_t* query_indices; /* [num_queries]                         */
  uint8_t* queries;        /* [num_queries][mlh_fri_query_bytes(L)]  */
} mlh_fri_proof;
uint64_t mlh_fri_query_bytes(uint32_t log_code);
/* FriProof::prove (fri/mod.rs:261-285); _gp: with the caller's gen_pows (above). */
mlh_status mlh_fri_prove(mlh_ctx* ctx, const void* dev_code, uint32_t log_code, mlh_transcript* tr,
                         mlh_fri_proof* proof);
mlh_status mlh_fri_prove_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                            const uint8_t gen_pows_1[16], uint32_t log_gen_pows, mlh_transcript* tr,
                            mlh_fri_proof* proof);
/* Wire format: serde + bincode 2 standard / little-endian / fixed-int encoding
 * of FriProof<Field128> (fri/mod.rs:239-249, 367-397; field.rs:40-64) -- the
 * bytes the reference's bincode::serde::encode_to_vec produces.  encode needs
 * query_indices (the Direction of every path level is bit i of the index);
 * decode fills commitments, queries, last_elem, last_random and (if non-NULL)
 * query_indices recovered from the directions; MLH_ERR_VERIFY if a path's
 * directions disagree with its index (the reference verifier rejects those). */
uint64_t mlh_fri_proof_encoded_size(const mlh_fri_proof* proof);
mlh_status mlh_fri_proof_encode(const mlh_fri_proof* proof, uint8_t* out, uint64_t cap);
mlh_status mlh_fri_proof_decode_header(const uint8_t* in, uint64_t len, uint32_t* log_code,
                                       uint32_t* num_queries);
mlh_status mlh_fri_proof_decode(const uint8_t* in, uint64_t len, mlh_fri_proof* proof);
/* FriProof::verify (fri/mod.rs:287-340), host side; MLH_ERR_VERIFY if rejected. */
mlh_status mlh_fri_verify(const mlh_fri_proof* proof);

/* Batched open_query_at: nq records (layout above) for host indices idx[nq]. */
mlh_status mlh_fri_prover_open_queries(mlh_ctx* ctx, const mlh_fri_prover* p,
                                       const uint64_t* idx, uint32_t nq, uint8_t* out);

/* ---- sharded building blocks (one process per GPU) ------------------------
 * The reference is single-node CPU code with no distributed API; these are
 * the rank-local steps multilinear_amd/dist.py drives between torch.distributed
 * (RCCL) collectives.  A sharded vector of 2^log_n elements over P = 2^log_p
 * ranks uses a block-cyclic layout with block 2^log_s: local index l of rank
 * r holds global ((l >> log_s) << (log_s + log_p)) | (r << log_s) | (l mod 2^log_s).
 * The distributed NTT (Polynomial::ntt / reed_solomon, ntt/mod.rs:69-108)
 * takes the cyclic layout (log_s = 0) and produces log_s = log_n - 2 log_p. */
/* Cross-shard stage: dev_in/dev_out are [P][S], S = 2^(log_n - 2 log_p).
 * Forward: row g of dev_in is the chunk received from rank g (its local
 * length-N/P NTT with generator gen^P, chunk `rank`); dev_out row t holds
 * X[t N/P + rank S + jl].  inverse != 0: the reverse (row t in, row g out,
 * scaled by 1/P; the local inverse NTT supplies 1/(N/P)).  gen has order 2^log_n. */
mlh_status mlh_shard_ntt_cross(mlh_ctx* ctx, const void* dev_in, void* dev_out, uint32_t log_n,
                               uint32_t log_p, uint32_t rank, const uint8_t gen[16], int inverse);
/* fold_step's fold (fri/mod.rs:89-114) on a sharded layer of 2^log_local local
 * values (pairs l, l + n_local/2 are global pairs i, i + n/2 while the layer
 * spans >= 2 blocks per rank); k and log_domain are global. */
mlh_status mlh_shard_fri_fold(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local, uint32_t k,
                              uint32_t log_domain, const uint8_t r[16], void* dev_next,
                              uint32_t log_s, uint32_t log_p, uint32_t rank);
/* Fold, then hash the folded layer's local leaves and build its local tree
 * (dev_tree: mlh_merkle_layers_bytes(2^(log_local-2)) bytes).  Levels below
 * log_s are the global tree's; the caller combines the level-log_s nodes of
 * all ranks. */
mlh_status mlh_shard_fri_fold_commit(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                     uint32_t k, uint32_t log_domain, const uint8_t r[16],
                                     void* dev_next, void* dev_tree, uint32_t log_s,
                                     uint32_t log_p, uint32_t rank);
/* Merkle::open / batch_open (merkle_tree/mod.rs:31-58, :134-175) on any device
 * tree of `leaves` leaves (mlh_merkle_commit*, level order): for each
 * host_idx[q] the log2(leaves) sibling digests, bottom-up, into host out
 * (nq * 32 * log2(leaves) bytes).  Direction of level i is Right iff bit i of
 * the index is 0.  MLH_ERR_INVALID for an index >= leaves (the reference
 * returns None).  The opened value is the caller's item (column) itself. */
mlh_status mlh_merkle_open(mlh_ctx* ctx, const void* dev_layers, uint64_t leaves,
                           const uint64_t* host_idx, uint32_t nq, uint8_t* out);
/* MerkleInclusionPath::verify / batch_verify (merkle_tree/mod.rs:216-293),
 * host side: value = the leaf bytes (batch_verify: the column items
 * concatenated), sibs = depth digests, dirs bit i = 1 for Direction::Left.
 * MLH_OK, MLH_ERR_VERIFY (IncompatibleHash) or MLH_ERR_VERIFY_INDEX
 * (IncompatibleIndex), checked in that order as the reference does. */
mlh_status mlh_merkle_verify(const uint8_t* value, uint64_t value_len, const uint8_t* sibs,
                             uint32_t depth, uint64_t dirs, const uint8_t root[32], uint64_t index);
/* Merkle::open (merkle_tree/mod.rs:31-58) on a local pair tree: for each
 * local leaf idx[q]: values[idx], values[idx + n/2], then the sibling digests
 * of levels 0..levels-1.  out: nq * 32 * (1 + levels) bytes (host). */
mlh_status mlh_merkle_open_pairs(mlh_ctx* ctx, const void* dev_values, uint32_t log_n,
                                 const void* dev_tree, uint32_t levels, const uint64_t* idx,
                                 uint32_t nq, uint8_t* out);

/* Device-resident Fiat-Shamir for sharded loops: the transcript state lives
 * in a mlh_device_transcript_bytes() device buffer (same bytes as the host
 * SHA-256 state); absorb reads from HBM and optionally writes
 * next_challenge() (16 B) to HBM, where the *_dr steps read it. */
uint64_t mlh_device_transcript_bytes(void);
mlh_status mlh_transcript_to_device(mlh_ctx* ctx, const mlh_transcript* tr, void* dev_state);
mlh_status mlh_transcript_from_device(mlh_ctx* ctx, const void* dev_state, mlh_transcript* tr);
mlh_status mlh_device_transcript_absorb(mlh_ctx* ctx, void* dev_state, const void* dev_src,
                                        uint32_t n, void* dev_challenge);
/* final fold's two values: flag (u32) = not an RS code, absorb LE16(v0), last = v0 */
mlh_status mlh_device_fri_last(mlh_ctx* ctx, const void* dev_vals2, void* dev_state,
                               void* dev_flag, void* dev_last);
/* mlh_shard_fri_fold(_commit) with the challenge read from HBM (dev_r, 16 B). */
mlh_status mlh_shard_fri_fold_dr(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                 uint32_t k, uint32_t log_domain, const void* dev_r,
                                 void* dev_next, uint32_t log_s, uint32_t log_p, uint32_t rank);
mlh_status mlh_shard_fri_fold_commit_dr(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                        uint32_t k, uint32_t log_domain, const void* dev_r,
                                        void* dev_next, void* dev_tree, uint32_t log_s,
                                        uint32_t log_p, uint32_t rank);
/* Cross-rank top of a sharded tree: dev_gathered = [P][per_rank] subtree roots
 * (all-gathered); dev_levels receives the tree over the P*per_rank nodes in
 * global order (t*P + h), level 0 first, root last: (2*P*per_rank - 1) x 32 B. */
mlh_status mlh_merkle_top(mlh_ctx* ctx, const void* dev_gathered, uint32_t P, uint64_t per_rank,
                          void* dev_levels);

/* Device-resident sumcheck steps: round sums written to HBM (2 x 16 B), the
 * challenge read from HBM; mlh_device_sumcheck_round adds npairs (s1, s2)
 * pairs (e.g. one per rank, all-gathered), interpolates, absorbs (c1, c2)
 * into the device transcript, writes c1 c2 and r, and updates the claim. */
mlh_status mlh_sumcheck_sums_dev(mlh_ctx* ctx, const void* dev_matrix, const void* dev_delta,
                                 uint32_t log_height, void* dev_sums);
mlh_status mlh_sumcheck_fold_sums_dr(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                     uint32_t log_height, const void* dev_r, void* dev_sums);
mlh_status mlh_sumcheck_fold_dr(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                uint32_t log_height, const void* dev_r);
mlh_status mlh_device_sumcheck_round(mlh_ctx* ctx, const void* dev_sum_pairs, uint32_t npairs,
                                     void* dev_prev, void* dev_state, void* dev_poly_out,
                                     void* dev_r_out);

/* ---- batched FRI / batched PCS (src/fri/batched_fri.rs, batched_pcs.rs) ----
 * m codes (or MLEs) stored back to back on the device: item j at j * size.
 * fingerprint(r, c_0..c_{m-1}) = Horner = sum_j c_j r^(m-1-j) (batched_fri.rs:30-38). */
typedef struct mlh_batched_fri_proof {
  uint32_t log_code;    /* L = log2(code length)                            */
  uint32_t num_codes;   /* m                                               */
  uint32_t num_trees;   /* inner FRI commitments: L - 2                    */
  uint32_t num_queries; /* MLH_NUM_QUERIES                                 */
  uint8_t batch_commitment[32];
  uint8_t* commitments; /* [num_trees][32]                                 */
  uint8_t last_elem[16];
  uint8_t last_random[32];
  uint64_t* query_indices; /* [num_queries] (optional)                     */
  uint8_t* queries;        /* [num_queries][mlh_batched_fri_query_bytes]   */
} mlh_batched_fri_proof;
/* Query record: the opened batch column (m x 32 B RS pairs, code order) and
 * its L-1 batch-tree siblings, then the inner QueryProof: for inner tree
 * t = 0..L-3 the pair (32 B) and its L-2-t siblings (directions = index bits). */
uint64_t mlh_batched_fri_query_bytes(uint32_t log_code, uint32_t num_codes);
/* BatchedFriProof::prove (batched_fri.rs:280-311). */
mlh_status mlh_batched_fri_prove(mlh_ctx* ctx, const void* dev_codes, uint32_t num_codes,
                                 uint32_t log_code, mlh_transcript* tr,
                                 mlh_batched_fri_proof* proof);
/* BatchedFriProof::verify (batched_fri.rs:313-388), host side. */
mlh_status mlh_batched_fri_verify(const mlh_batched_fri_proof* proof);
/* BatchedFriProverData step by step (batched_fri.rs:9-224), the transcript on
 * the host: what BatchedFriProverData::fold (:178-205) and BatchedPCSProverData
 * (batched_pcs.rs:80-125) call.
 *  - init (:41-98): batch layer of the m codes' RS pairs (dev_codes = the codes
 *    back to back, 2^log_code each, kept by the caller while the prover lives),
 *    absorb its root, fingerprint_r = next_challenge(), absorb LE16 of it;
 *  - fold_step_gp = batched_fold_step(&mut self, gen_pows, r, transcript)
 *    (:100-176): fingerprinted pairs folded with k = 0 and twiddle
 *    gen_pows[len - i], then the folded layer's tree (or, at 4 elements, the
 *    last element) into fri_data, and its root (last element) absorbed; a
 *    second call is MLH_ERR_INVALID (the reference would fold the batch layer
 *    again);
 *  - inner = &mut self.fri_data: the FriProverData whose fold_step(gen_pows, k,
 *    r, tr) the reference calls for k >= 1 (:200) -- pass it to
 *    mlh_fri_prover_fold_step(_gp), _roots, _last_element, _open_query(ies);
 *    owned by the batched prover (do not destroy it);
 *  - open_query = open_query_at (:207-224): one record in the
 *    mlh_batched_fri_query_bytes layout (inner part zero where fri_data has
 *    no tree yet). */
typedef struct mlh_batched_fri_prover mlh_batched_fri_prover;
mlh_status mlh_batched_fri_prover_init(mlh_ctx* ctx, const void* dev_codes, uint32_t num_codes,
                                       uint32_t log_code, mlh_transcript* tr,
                                       mlh_batched_fri_prover** out);
mlh_status mlh_batched_fri_prover_fold_step_gp(mlh_ctx* ctx, mlh_batched_fri_prover* bp,
                                               const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                               const uint8_t r[16], mlh_transcript* tr);
mlh_fri_prover* mlh_batched_fri_prover_inner(mlh_batched_fri_prover* bp);
mlh_status mlh_batched_fri_prover_batch_root(const mlh_batched_fri_prover* bp, uint8_t out[32]);
mlh_status mlh_batched_fri_prover_fingerprint_r(const mlh_batched_fri_prover* bp, uint8_t out[16]);
mlh_status mlh_batched_fri_prover_open_query(mlh_ctx* ctx, const mlh_batched_fri_prover* bp,
                                             uint64_t index, uint8_t* out);
void mlh_batched_fri_prover_destroy(mlh_batched_fri_prover* bp);
typedef struct mlh_batched_pcs_proof {
  mlh_batched_fri_proof fri;
  uint8_t* sumcheck_polys; /* [n_vars][2][16] */
} mlh_batched_pcs_proof;
/* BatchedPCSProof::prove (batched_pcs.rs:127-180): dev_evals = num_polys MLEs
 * of 2^n_vars evals; claim = (inputs[n_vars], outputs[num_polys]) LE16 each. */
mlh_status mlh_batched_pcs_prove(mlh_ctx* ctx, const void* dev_evals, uint32_t num_polys,
                                 uint32_t n_vars, const uint8_t* inputs, const uint8_t* outputs,
                                 mlh_transcript* tr, mlh_batched_pcs_proof* proof);
/* BatchedPCSProof::verify (batched_pcs.rs:182-250), host side. */
mlh_status mlh_batched_pcs_verify(const mlh_batched_pcs_proof* proof, uint32_t n_vars,
                                  const uint8_t* inputs, const uint8_t* outputs,
                                  mlh_transcript* tr);

/* ---- transcript (src/transcript.rs), host side --------------------------- */
mlh_status mlh_transcript_create(mlh_transcript** out);
mlh_status mlh_transcript_clone(const mlh_transcript* t, mlh_transcript** out);
void mlh_transcript_destroy(mlh_transcript* t);
mlh_status mlh_transcript_absorb(mlh_transcript* t, const uint8_t* bytes, uint64_t len); /* :31 */
mlh_status mlh_transcript_random(const mlh_transcript* t, uint8_t out[32]);             /* :23 */
mlh_status mlh_transcript_next_challenge(mlh_transcript* t, uint8_t out[16]);          /* :35 */

/* ---- multilinear polynomials and sumcheck -------------------------------- */
/* MultilinearPolynomialEvals::to_coefficient (polynomials.rs:150-163), in place. */
mlh_status mlh_mle_to_coefficient(mlh_ctx* ctx, void* dev_evals, uint32_t log_n);
/* MultilinearPolynomial::to_evaluation (polynomials.rs:111-124), in place. */
mlh_status mlh_mle_to_evaluation(mlh_ctx* ctx, void* dev_coeffs, uint32_t log_n);
/* delta table of SumcheckTables::build_tables_for_pcs (sumcheck.rs:128-145,
 * Mask::evaluate evaluation.rs:51-73): out[idx] = prod_i (bit_i(idx) ?
 * p[n-1-i] : 1-p[n-1-i]); host_points: n elements. */
mlh_status mlh_eq_table(mlh_ctx* ctx, const uint8_t* host_points, uint32_t n, void* dev_out);
/* MultilinearPolynomialEvals::evaluate (polynomials.rs:165-187). */
mlh_status mlh_mle_evaluate(mlh_ctx* ctx, const void* dev_evals, uint32_t n,
                            const uint8_t* host_args, uint8_t out[16]);
/* MultilinearPolynomial::evaluate (polynomials.rs:126-146), coefficient form:
 * sum_pos coeffs[pos] * prod_{bit b of pos set} args[n-1-b]. */
mlh_status mlh_mle_coeffs_evaluate(mlh_ctx* ctx, const void* dev_coeffs, uint32_t n,
                                   const uint8_t* host_args, uint8_t out[16]);
/* Polynomial::evaluate (ntt/mod.rs:61-67, polynomials.rs:9-14): Horner's
 * value sum_i coeffs[i] x^i of n device coefficients at host x (canonical);
 * n = 0 gives 0. */
mlh_status mlh_poly_evaluate(mlh_ctx* ctx, const void* dev_coeffs, uint64_t n, const uint8_t x[16],
                             uint8_t out[16]);
/* Trace::evaluate (constraint_system/evaluation.rs:31-48): the row-major
 * 2^log_height x width trace (dev_matrix, element (i, j) at i*width + j) as
 * width MLEs evaluated at the log_height host points (big-endian, Mask order):
 * out[j] = sum_i Mask{i}(points) * matrix[i*width + j]; out: 16*width bytes. */
mlh_status mlh_trace_evaluate(mlh_ctx* ctx, const void* dev_matrix, uint32_t log_height,
                              uint32_t width, const uint8_t* host_points, uint8_t* out);
/* SumcheckTables::partial_sum (sumcheck.rs:204-232), composition x[0]
 * (multilinear_pcs.rs:56), at X = 1 and X = 2: out = s1 ‖ s2.
 * Tables have 2^log_height elements. */
mlh_status mlh_sumcheck_partial_sums(mlh_ctx* ctx, const void* dev_matrix, const void* dev_delta,
                                     uint32_t log_height, uint8_t out[32]);
/* SumcheckTables::fold (sumcheck.rs:234-247), in place: height 2^log_height
 * -> 2^(log_height-1) (first half). */
mlh_status mlh_sumcheck_fold(mlh_ctx* ctx, void* dev_matrix, void* dev_delta, uint32_t log_height,
                             const uint8_t r[16]);
/* fold followed by the next round's partial sums, one HBM pass. */
mlh_status mlh_sumcheck_fold_and_sums(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                      uint32_t log_height, const uint8_t r[16], uint8_t out[32]);
/* SumcheckTables::compute_sumcheck_polynomials (sumcheck.rs:77-102) for the
 * PCS composition (x[0], total degree 2): log_height rounds; per round the
 * two nonzero coefficients (c1, c2) go to polys_out[round][2][16] and the
 * challenge to rs_out[round][16].  Tables are folded in place. */
mlh_status mlh_sumcheck_prove(mlh_ctx* ctx, void* dev_matrix, void* dev_delta, uint32_t log_height,
                              const uint8_t sum[16], mlh_transcript* tr, uint8_t* polys_out,
                              uint8_t* rs_out);
/* SumcheckTables::build_tables_for_pcs (sumcheck.rs:128-145) followed by
 * compute_sumcheck_polynomials (:77-102), with the delta table = eq(points)
 * never materialised at full size: it stays c_k * eq(p_k..p_{L-1}) (a running
 * scalar times a two-level factored table) until it has 2^12 entries.  Same
 * outputs as mlh_eq_table + mlh_sumcheck_prove; half the HBM traffic.
 * dev_evals: the MLE (2^log_height elements).  dev_work (2^(log_height-1)
 * elements) receives the folded matrix (the first half of the table as
 * SumcheckTables::fold leaves it) and dev_evals is not modified -- the
 * matrix clone of build_tables_for_pcs is never made; dev_work = NULL folds
 * dev_evals in place.  host_points: log_height elements; delta_out
 * (optional): the fully folded delta. */
mlh_status mlh_sumcheck_prove_eq(mlh_ctx* ctx, const void* dev_evals, void* dev_work,
                                 uint32_t log_height, const uint8_t* host_points,
                                 const uint8_t sum[16], mlh_transcript* tr, uint8_t* polys_out,
                                 uint8_t* rs_out, uint8_t* delta_out);

/* ---- multilinear PCS (src/fri/multilinear_pcs.rs) ------------------------ */
typedef struct mlh_pcs_proof {
  mlh_fri_proof fri;
  uint8_t* sumcheck_polys; /* [n_vars][2][16] nonzero coefficients c1, c2 */
} mlh_pcs_proof;
/* PCSProof::prove (multilinear_pcs.rs:90-136): dev_evals (2^n_vars elements)
 * is not modified; host_inputs: n_vars points; output: the claimed value. */
mlh_status mlh_pcs_prove(mlh_ctx* ctx, const void* dev_evals, uint32_t n_vars,
                         const uint8_t* host_inputs, const uint8_t output[16], mlh_transcript* tr,
                         mlh_pcs_proof* proof);
/* PCSProof::verify (multilinear_pcs.rs:138-190), host side. */
mlh_status mlh_pcs_verify(const mlh_pcs_proof* proof, uint32_t n_vars, const uint8_t* host_inputs,
                          const uint8_t output[16], mlh_transcript* tr);

/* ---- multi-GPU: one process per GPU -------
 * The reference has no distributed API; these run its NTT / reed_solomon /
 * FriProof::prove / sumcheck on P = 2^p ranks.  Exchanges go through a
 * transport: the built-in one is RCCL over xGMI (mlh_comm: rank 0 calls
 * mlh_comm_unique_id and sends the 128 bytes to the other ranks out of band,
 * every rank calls mlh_comm_create); a caller may supply its own (e.g. over
 * host memory; host_side = 1 makes the library drain its stream before each
 * call).  Every rank calls the same entry point with its shard; collectives
 * are enqueued on the context stream.
 * Layout of a sharded 2^log_n vector: block-cyclic with block 2^log_s, local
 * index l of rank r = global ((l >> log_s) << (log_s + p)) | (r << log_s) |
 * (l mod 2^log_s); "cyclic" = log_s 0. */
typedef int (*mlh_all_to_all_fn)(void* user, const void* dev_send, void* dev_recv,
                                 uint64_t bytes_per_rank, void* hip_stream);
typedef int (*mlh_all_gather_fn)(void* user, const void* dev_send, void* dev_recv, uint64_t bytes,
                                 void* hip_stream);
typedef struct mlh_transport {
  uint32_t world;     /* P, a power of two <= 16                                */
  uint32_t rank;      /* this process                                           */
  uint32_t host_side; /* 1: callbacks complete on the host (stream drained first) */
  void* user;
  /* chunk i (bytes_per_rank) of dev_send goes to rank i; chunk i of dev_recv came from rank i */
  mlh_all_to_all_fn all_to_all;
  /* dev_recv = every rank's dev_send (bytes each), in rank order */
  mlh_all_gather_fn all_gather;
} mlh_transport;
typedef struct mlh_comm mlh_comm;
mlh_status mlh_comm_unique_id(uint8_t out[128]);
mlh_status mlh_comm_create(mlh_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t id[128],
                           mlh_comm** out);
void mlh_comm_destroy(mlh_comm* comm);
mlh_status mlh_comm_transport(mlh_comm* comm, mlh_transport* out);
/* What RCCL itself reports for the communicator (ncclCommCount,
 * ncclCommUserRank, ncclCommCuDevice): the ranks it connected, this rank, and
 * its device -- the self-check a multi-GPU run prints. */
mlh_status mlh_comm_info(mlh_comm* comm, uint32_t* count, uint32_t* rank, int* device);
/* Transport pre-flight (no reference counterpart): one all-to-all of
 * P x bytes_per_rank and one all-gather of bytes_per_rank through `tp`, each
 * word a function of (source rank, destination rank, position), checked on the
 * device.  *mismatches = the words this rank received wrong (0 on a sound
 * transport); *ms (optional) = the two collectives' duration on the context
 * stream.  Run it before the first data-path collective of a multi-GPU job. */
mlh_status mlh_comm_preflight(mlh_ctx* ctx, const mlh_transport* tp, uint64_t bytes_per_rank,
                              uint64_t* mismatches, float* ms);
/* Polynomial::ntt / LagrangePolynomial::intt (ntt/mod.rs:69-173) of a 2^log_n
 * vector: forward takes the cyclic layout (2^log_n / P local elements) and
 * returns block 2^log_n / P^2; inverse != 0 the reverse.  One all-to-all. */
mlh_status mlh_sharded_ntt(mlh_ctx* ctx, const mlh_transport* tp, const void* dev_in, void* dev_out,
                           uint32_t log_n, const uint8_t gen[16], int inverse);
/* count sharded NTTs (or INTTs) of 2^log_n vectors, dev_in[i] -> dev_out[i]
 * with mlh_sharded_ntt's layouts, pipelined on two streams: the all-to-all of
 * transform i (and the local step after it) runs on the context's second
 * stream while the first local step of transform i + 1 runs on the context
 * stream.  On return the context stream is ordered after all of them.  This is
 * Polynomial::ntt (ntt/mod.rs:69-110) called on count polynomials in turn. */
mlh_status mlh_sharded_ntt_batch(mlh_ctx* ctx, const mlh_transport* tp, const void* const* dev_in,
                                 void* const* dev_out, uint32_t count, uint32_t log_n,
                                 const uint8_t gen[16], int inverse);
/* The same forward transforms with the rank digit fused into the last pass:
 * the local passes but the last, ONE all-to-all, one pass over the received
 * chunks -- three HBM passes per element instead of the local NTT's three plus
 * the cross-shard DFT's.  Input cyclic (rank g holds x[g + P m]);
 * output block-cyclic with block 2^(*log_s_out) (the plan's first digit minus
 * log2 P: 6 at 2^27 over 8 ranks), i.e. local l of rank r is global
 * ((l >> s) << (s + p)) | (r << s) | (l mod 2^s).  2 <= P <= 8; local size
 * >= 2^(13 - log2 P).  Pipelined on three streams like mlh_sharded_ntt_batch. */
mlh_status mlh_sharded_ntt_fused_batch(mlh_ctx* ctx, const mlh_transport* tp, const void* const* dev_in,
                                       void* const* dev_out, uint32_t count, uint32_t log_n,
                                       const uint8_t gen[16], uint32_t* log_s_out);
/* reed_solomon (fri/mod.rs:19-28): 2^log_n coefficients in the cyclic layout,
 * gen of order 2^(log_n + 1) -> the codeword in block 2^(log_n + 1) / P^2. */
mlh_status mlh_sharded_reed_solomon(mlh_ctx* ctx, const mlh_transport* tp, const void* dev_coeffs,
                                    uint32_t log_n, const uint8_t gen[16], void* dev_code);
/* commit_rs_code (fri/mod.rs:45-55) + Merkle::commit (merkle_tree/mod.rs:65-85)
 * of a 2^log_code codeword in the block 2^log_code / P^2 layout: local leaves
 * and subtrees, one all-gather of the subtree roots, the top levels on every
 * rank; root_out (host) = the root of the natural-order codeword's tree. */
mlh_status mlh_sharded_commit_rs_code(mlh_ctx* ctx, const mlh_transport* tp, const void* dev_code,
                                      uint32_t log_code, uint8_t root_out[32]);
/* FriProof::prove (fri/mod.rs:261-285) of a 2^log_code codeword in the block
 * 2^log_code / P^2 layout (mlh_sharded_reed_solomon's output); layers below
 * 2^gather_log entries are gathered and finished replicated (16 is a good
 * value).  Every rank returns the same proof: byte-identical to mlh_fri_prove
 * of the natural-order codeword. */
mlh_status mlh_sharded_fri_prove(mlh_ctx* ctx, const mlh_transport* tp, const void* dev_code,
                                 uint32_t log_code, uint32_t gather_log, mlh_transcript* tr,
                                 mlh_fri_proof* proof);
/* build_tables_for_pcs's delta (sumcheck.rs:128-145) in the cyclic layout:
 * rank r gets delta[l P + r], l < 2^(n - p). */
mlh_status mlh_sharded_eq_table(mlh_ctx* ctx, const mlh_transport* tp, const uint8_t* points,
                                uint32_t n, void* dev_out);
/* compute_sumcheck_polynomials (sumcheck.rs:77-102), composition x[0], of
 * tables in the cyclic layout; polys_out [n][2][16], rs_out [n][16] as
 * mlh_sumcheck_prove.  The local tables are folded in place while they hold
 * >= 2 entries (the last log2 P rounds fold gathered copies); on return entry
 * 0 of every rank's dev_m / dev_d holds the fully folded m(r) / d(r), the
 * length-1 tables the reference ends with.  The RCCL transport (mlh_comm) at
 * P > 1 has run only on the driver's multi-GPU node; the tests drive these
 * entry points at P > 1 through a host-side transport. */
mlh_status mlh_sharded_sumcheck_prove(mlh_ctx* ctx, const mlh_transport* tp, void* dev_m, void* dev_d,
                                      uint32_t n, const uint8_t sum[16], mlh_transcript* tr,
                                      uint8_t* polys_out, uint8_t* rs_out);

/* ---- device timing helpers (bench / profiling) --------------------------- */
/* Kernel timer: while enabled, the NTT pass launches are bracketed by HIP
 * events on the context stream -- those of every transform for on = 1, of
 * every on-th transform for on > 1 (each timing event costs the stream a few
 * microseconds; sampling keeps that out of a throughput measurement);
 * mlh_profile_get (synchronising) returns the launch count and summed
 * milliseconds of the bracketed launches for a kernel label such as
 * "ntt_pass<8,0,0>" (radix log2, last pass, zero-padded input). */
mlh_status mlh_profile_enable(mlh_ctx* ctx, int on);
mlh_status mlh_profile_reset(mlh_ctx* ctx);
mlh_status mlh_profile_get(mlh_ctx* ctx, const char* label, uint64_t* count, double* total_ms);
/* Time `iters` forward NTTs of 2^log_n on the context stream with HIP events
 * (dev_buf is transformed in place); returns the mean ms per NTT. */
mlh_status mlh_bench_ntt(mlh_ctx* ctx, void* dev_buf, uint32_t log_n, uint32_t iters,
                         float* ms_out);

#ifdef __cplusplus
}
#endif
#endif /* MLHIP_H */
