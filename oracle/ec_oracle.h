/*
 * ec_oracle.h — CPU restatement of the ec-cpp NPB Reed-Solomon codec.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity *checker*: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (erasure-coding-crust_amd/) never links or calls it.
 *
 * Pinned against: (1) the reference's golden tables
 * (include/ec-cpp/table_f2e16.hpp, via tests/golden/tables.json digests) and
 * (2) outputs of the reference ec-cpp itself, compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/ (the tests/golden JSON files
 * produced by tests/golden/make_golden.py).
 *
 * Every function names the reference file:line it restates.
 */
#ifndef EC_ORACLE_H
#define EC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes = ec_cpp::Error order (include/ec-cpp/errors.hpp:13-24), +1; 0 = ok */
enum {
  ECO_OK = 0,
  ECO_ARGS_MUST_BE_POW2 = 1,
  ECO_WANTED_SHARD_COUNT_TOO_LOW = 2,
  ECO_WANTED_SHARD_COUNT_TOO_HIGH = 3,
  ECO_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW = 4,
  ECO_PAYLOAD_SIZE_IS_ZERO = 5,
  ECO_TOO_MANY_VALIDATORS = 6,
  ECO_NOT_ENOUGH_VALIDATORS = 7,
  ECO_NEED_MORE_SHARDS = 8,
  ECO_INCONSISTENT_SHARD_LENGTHS = 9,
  ECO_EMPTY_SHARD = 10,
};

/* tables (f2e16.hpp:48-84, additive_fft.hpp:47-97) */
const uint16_t *eco_log_table(void);
const uint16_t *eco_exp_table(void);
const uint16_t *eco_log_walsh_table(void);
const uint16_t *eco_skews(void); /* 65535 entries */

uint16_t eco_mul(uint16_t x, uint16_t log_c);              /* additive_fft.hpp:21-33 */
void eco_walsh(uint16_t *data, size_t size);              /* walsh.hpp:15-39 */
void eco_inverse_afft(uint16_t *data, size_t size, size_t index); /* additive_fft.hpp:99-119 */
void eco_afft(uint16_t *data, size_t size, size_t index);         /* additive_fft.hpp:121-141 */
void eco_formal_derivative(uint16_t *cos, size_t size);    /* poly_encoder.hpp:195-215 */

/* parameters: ec-cpp.cpp:15-37 + reed-solomon.hpp:24-45 */
int eco_recovery_threshold(size_t n_validators, size_t *threshold);
int eco_params(size_t n_validators, size_t *n, size_t *k);
size_t eco_shard_len(size_t k, size_t payload_len); /* reed-solomon.hpp:191-196 */

/* encode: reed-solomon.hpp:47-81.  shards = wanted_n * shard_len bytes, shard-major */
int eco_encode(size_t n_validators, const uint8_t *payload, size_t len,
               uint8_t *shards, size_t shards_cap);

/* error locator: poly_encoder.hpp:90-116 (direct 65536-point form).
 * erased[i] != 0 for i < n_received means shard i is missing; indices
 * >= n_received count as erased.  out: 65536 log-multipliers. */
void eco_error_poly(const uint8_t *erased, size_t n_received, size_t n,
                    uint16_t *out);
/* exact O(n log n) folded form of the same residues mod 65535 (first n) */
void eco_error_poly_folded(const uint8_t *erased, size_t n_received, size_t n,
                           uint16_t *out);

/* reconstruct: reed-solomon.hpp:83-134.  shards[i] == NULL or lens[i]==0 means
 * missing.  out must hold shard_len/2*2*k bytes; *out_len receives it. */
int eco_reconstruct(size_t n_validators, const uint8_t *const *shards,
                    const size_t *lens, size_t n_received, uint8_t *out,
                    size_t out_cap, size_t *out_len);

/* reed-solomon.hpp:143-179 */
int eco_reconstruct_from_systematic(size_t n_validators,
                                    const uint8_t *const *chunks,
                                    const size_t *lens, size_t count,
                                    uint8_t *out, size_t out_cap,
                                    size_t *out_len);

#ifdef __cplusplus
}
#endif
#endif
