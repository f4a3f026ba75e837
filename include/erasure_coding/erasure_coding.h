/*
 * erasure_coding.h — drop-in C ABI of qdrvm/erasure-coding-crust, served by the
 * MI355X (gfx950) HIP implementation in erasure-coding-crust_amd/.
 *
 * The reference generates this header with cbindgen from src/erasure_coding.rs
 * (build.rs:7-12, cbindgen.toml: language=C, style=Both, cpp_compat=true,
 * rename_variants=QualifiedScreamingSnakeCase).  The layout below reproduces
 * that output: same type names, field order, enum discriminants and function
 * signatures (c_ulong == unsigned long on LP64).  Link against
 * liberasure_coding_crust.so (this repo) instead of the Rust cdylib.
 *
 * Results are bit-exact with ec-cpp (/root/reference/ec-cpp/ec-cpp.cpp).
 */
#ifndef _NOVELPOLY_REED_SOLOMON_CRUST_INCLUDE_GUARD_H_
#define _NOVELPOLY_REED_SOLOMON_CRUST_INCLUDE_GUARD_H_

#include <stdarg.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>

/* Errors in erasure coding.  (src/erasure_coding.rs:10-46) */
typedef enum NPRSResult_Tag {
  NPRS_RESULT_OK,                        /* No error */
  NPRS_RESULT_TOO_MANY_VALIDATORS,       /* too many validators */
  NPRS_RESULT_NOT_ENOUGH_VALIDATORS,     /* cannot encode for zero or one validator */
  NPRS_RESULT_WRONG_VALIDATOR_COUNT,     /* cannot reconstruct: wrong validator count */
  NPRS_RESULT_NOT_ENOUGH_CHUNKS,         /* not enough chunks present */
  NPRS_RESULT_TOO_MANY_CHUNKS,           /* too many chunks present */
  NPRS_RESULT_NON_UNIFORM_CHUNKS,        /* chunks not of uniform length or empty */
  NPRS_RESULT_UNEVEN_LENGTH,             /* odd shard byte-length */
  NPRS_RESULT_CHUNK_INDEX_OUT_OF_BOUNDS, /* chunk index out of bounds */
  NPRS_RESULT_BAD_PAYLOAD,               /* bad payload */
  NPRS_RESULT_INVALID_BRANCH_PROOF,      /* invalid branch proof */
  NPRS_RESULT_BRANCH_OUT_OF_BOUNDS,      /* branch out of bounds */
  NPRS_RESULT_UNKNOWN_RECONSTRUCTION,    /* unknown error */
  NPRS_RESULT_UNKNOWN_CODE_PARAM,        /* unknown error */
} NPRSResult_Tag;

typedef struct NPRSResult_ChunkIndexOutOfBounds_Body {
  unsigned long chunk_index;  /* index of invalid chunk */
  unsigned long n_validators; /* number of validators */
} NPRSResult_ChunkIndexOutOfBounds_Body;

typedef struct NPRSResult {
  NPRSResult_Tag tag;
  union {
    NPRSResult_ChunkIndexOutOfBounds_Body chunk_index_out_of_bounds;
  };
} NPRSResult;

/* Represent the data array  (src/erasure_coding.rs:49-53) */
typedef struct DataBlock {
  uint8_t *array;
  unsigned long length;
} DataBlock;

/* Represent chunk of the data  (src/erasure_coding.rs:56-60) */
typedef struct Chunk {
  struct DataBlock data;
  unsigned long index;
} Chunk;

/* Represent the array of chunks  (src/erasure_coding.rs:63-67) */
typedef struct ChunksList {
  struct Chunk *data;
  unsigned long count;
} ChunksList;

#ifdef __cplusplus
extern "C" {
#endif

/* Obtain a threshold of chunks that should be enough to recover the data.
 * Replaces src/erasure_coding.rs:106-120.  Host-only (no GPU needed). */
struct NPRSResult ECCR_get_recovery_threshold(unsigned long validators_number,
                                              unsigned long *threshold_out);

/* Cleans the data block.  Replaces src/erasure_coding.rs:125-129 (free()). */
void ECCR_deallocate_data_block(struct DataBlock *data);

/* Cleans the data in chunk.  Replaces src/erasure_coding.rs:134-137. */
void ECCR_deallocate_chunk(struct Chunk *data);

/* Cleans the data allocated for the chunk list.  Replaces
 * src/erasure_coding.rs:142-153: frees every shard buffer and the array. */
void ECCR_deallocate_chunk_list(struct ChunksList *chunk_list);

/* Copies the 65,535 AFFT skew factors.  Replaces src/erasure_coding.rs:160-169.
 * Host-only. */
struct NPRSResult ECCR_AFFT_Table(uint16_t (*output)[65535]);

/* Encode + reconstruct(all chunks), timed in microseconds (host-to-host,
 * including H2D/D2H).  Replaces src/erasure_coding.rs:174-217. */
struct NPRSResult ECCR_Test_MeasurePerformance(const struct DataBlock *message,
                                               unsigned long n_validators,
                                               unsigned long *usEncoding,
                                               unsigned long *usDecoding);

/* Obtain erasure-coded chunks, one for each validator.  Replaces
 * src/erasure_coding.rs:224-267.  The library allocates output->data
 * (n_validators Chunks, index = position) and one malloc'd buffer per shard;
 * free with ECCR_deallocate_chunk_list.  An empty payload returns
 * NPRS_RESULT_BAD_PAYLOAD (the reference panics). */
struct NPRSResult ECCR_obtain_chunks(unsigned long validators_number,
                                     const struct DataBlock *message,
                                     struct ChunksList *output);

/* Reconstruct from the k systematic chunks (index < k).  Replaces
 * src/erasure_coding.rs:277-334.  Output is zero-padded; truncate to the
 * payload length.  Free with ECCR_deallocate_data_block. */
struct NPRSResult ECCR_reconstruct_from_systematic(unsigned long validators_number,
                                                   const struct ChunksList *input_chunks,
                                                   struct DataBlock *outdata);

/* Reconstruct data from a set of chunks (positional by Chunk.index; null or
 * empty chunks are skipped; only the first n_validators list entries are
 * read).  Replaces src/erasure_coding.rs:344-409.  Output is
 * shard_len * k bytes, zero-padded; free with ECCR_deallocate_data_block. */
struct NPRSResult ECCR_reconstruct(unsigned long validators_number,
                                   const struct ChunksList *input_chunks,
                                   struct DataBlock *outdata);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* _NOVELPOLY_REED_SOLOMON_CRUST_INCLUDE_GUARD_H_ */
