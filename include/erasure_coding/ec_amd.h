/*
 * ec_amd.h — MI355X device-resident batch extension of the erasure_coding.h
 * C ABI.  These are NEW symbols (the nine ECCR_* entry points are unchanged).
 *
 * All pointers named d_* are device pointers on the codec's device; `stream`
 * is a hipStream_t (NULL = the legacy default stream).  Calls are asynchronous
 * on `stream` and the caller owns every buffer it passes.  Shapes that need
 * device scratch (k = 1024 encodes, the fast reconstructs' per-payload gather
 * order (4 n bytes per payload; n = 2048 / 4096 add an 80 KB output-table
 * image per payload), n > 4096 generic kernels,
 * ECCR_AMD_error_locator / ECCR_AMD_dedup_patterns with batch > 1) use, in the
 * plain calls, a scratch buffer private to (device, stream): the first call of
 * a larger shape on a stream allocates it (hipMalloc, after synchronising that
 * stream if a smaller one is replaced); afterwards the plain calls allocate,
 * record and wait on nothing, and calls on different streams never wait on
 * each other.  Host threads may issue plain calls on the same stream
 * concurrently: each call holds that stream's scratch until it has enqueued
 * all its kernels, so the calls run one after the other on the stream.  A
 * stream keeps its largest scratch until ECCR_AMD_release_stream_scratch or
 * until more than 64 streams of the device have one: then the least recently
 * used is evicted, and evicted buffers are freed 16 at a time, after a
 * device-wide synchronisation (which waits for work on every stream of the
 * device), at the start of a plain call on a stream that is not being
 * captured.  That synchronisation invalidates a hipGraph capture another
 * thread has open in global mode (hipStreamCaptureModeGlobal) at that moment:
 * programs that capture in global mode while more than 64 streams use the
 * plain calls should release retired streams' scratch with
 * ECCR_AMD_release_stream_scratch (outside any capture), use the *_ws calls,
 * or capture in thread-local / relaxed mode.  The *_ws variants take caller-owned scratch instead (size from
 * the matching *_workspace_bytes query) and never allocate.  Either form can
 * be captured into a hipGraph and replayed once the shape has run once on the
 * stream outside capture (the first call per (device, kernel) also sets a
 * kernel attribute and uploads the tables).  Results are bit-exact with ec-cpp:
 *   encode      == ReedSolomon::encode      (include/ec-cpp/reed-solomon.hpp:47-81)
 *   reconstruct == ReedSolomon::reconstruct (include/ec-cpp/reed-solomon.hpp:83-134)
 *   systematic  == ReedSolomon::reconstruct_from_systematic (:143-179)
 *
 * Layouts (one batch = `batch` independent payloads of the same length):
 *   payloads   : [batch][payload_stride] bytes, payload_len used
 *   shards     : [batch][n_validators][shard_stride] bytes, shard_len used
 *   present    : [batch][n] bytes, 1 = shard present (indices >= n_validators
 *                are always treated as erased)
 *   err_log    : [batch][n] uint16 log-domain erasure-locator multipliers
 *                (poly_encoder.hpp:90-116), produced by ECCR_AMD_error_locator
 *   out        : [batch][out_stride] bytes, shard_len * k used (zero-padded
 *                past payload_len, as the reference)
 */
#ifndef ERASURE_CODING_EC_AMD_H_
#define ERASURE_CODING_EC_AMD_H_

#include "erasure_coding.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Code parameters for n_validators (ec-cpp.cpp:15-37): n = po2 >= nv,
 * k = po2 <= threshold.  Host-only. */
struct NPRSResult ECCR_AMD_code_params(unsigned long n_validators, unsigned long *n,
                                       unsigned long *k, unsigned long *threshold);

/* shard_len(payload_len) = ceil(ceil(len/2)/k)*2 (reed-solomon.hpp:191-196). */
unsigned long ECCR_AMD_shard_len(unsigned long n_validators, unsigned long payload_len);

/* Number of visible HIP devices (0 if none / runtime unusable). */
int ECCR_AMD_device_count(void);

/* Upload field tables and skews to the current device (idempotent). */
struct NPRSResult ECCR_AMD_init_device(void);

/* Device-resident batch encode. */
struct NPRSResult ECCR_AMD_encode_batch(unsigned long n_validators, const uint8_t *d_payloads,
                                        unsigned long payload_len, unsigned long payload_stride,
                                        unsigned long batch, uint8_t *d_shards,
                                        unsigned long shard_stride, void *stream);

/* Erasure-locator multipliers for a batch of erasure patterns, one row of
 * d_err_log per row of d_present.  With batch > 1, equal patterns are found on
 * the device (ECCR_AMD_dedup_patterns) and each distinct one is computed once,
 * then copied to the payloads that share it. */
struct NPRSResult ECCR_AMD_error_locator(unsigned long n_validators, const uint8_t *d_present,
                                         unsigned long batch, uint16_t *d_err_log,
                                         void *stream);

/* Device-resident batch reconstruct (needs ECCR_AMD_error_locator output).
 * The device path does not count shards: a payload with fewer than k present
 * shards yields unspecified bytes (never an out-of-bounds access).  The host
 * entry points (ECCR_reconstruct, ECCR_AMD_reconstruct_host_batch) check the
 * count and return NOT_ENOUGH_CHUNKS.  Missing shards' bytes are never read. */
struct NPRSResult ECCR_AMD_reconstruct_batch(unsigned long n_validators, const uint8_t *d_shards,
                                             unsigned long shard_len, unsigned long shard_stride,
                                             const uint8_t *d_present, const uint16_t *d_err_log,
                                             unsigned long batch, uint8_t *d_out,
                                             unsigned long out_stride, void *stream);

/* ---- caller-owned scratch (graph capture) ---------------------------------
 * Bytes of device scratch the batch calls above need for a shape (0 = none;
 * also 0 for invalid parameters, which the calls themselves report), and the
 * same calls with that scratch passed in: d_workspace 256-B aligned, at least
 * the queried size (else UNKNOWN_* and nothing is launched).  A workspace may
 * be shared by calls that are ordered on one stream.  Encode shapes with
 * k = 16 .. 1024 and n <= 4096 (n_validators 46 .. 4096) query 256 bytes
 * since round 5: a tile counter for their dynamic schedule.  A smaller (or NULL) workspace is accepted for those
 * shapes and runs them on a static schedule (a few percent slower), so a size
 * of 0 cached from an earlier release still works. */
unsigned long ECCR_AMD_encode_workspace_bytes(unsigned long n_validators,
                                              unsigned long payload_len, unsigned long batch);
unsigned long ECCR_AMD_error_locator_workspace_bytes(unsigned long n_validators,
                                                     unsigned long batch);
unsigned long ECCR_AMD_reconstruct_workspace_bytes(unsigned long n_validators,
                                                   unsigned long shard_len, unsigned long batch);
struct NPRSResult ECCR_AMD_encode_batch_ws(unsigned long n_validators, const uint8_t *d_payloads,
                                           unsigned long payload_len, unsigned long payload_stride,
                                           unsigned long batch, uint8_t *d_shards,
                                           unsigned long shard_stride, void *d_workspace,
                                           unsigned long workspace_bytes, void *stream);
struct NPRSResult ECCR_AMD_error_locator_ws(unsigned long n_validators, const uint8_t *d_present,
                                            unsigned long batch, uint16_t *d_err_log,
                                            void *d_workspace, unsigned long workspace_bytes,
                                            void *stream);
/* d_pattern as in ECCR_AMD_reconstruct_batch_patterns (NULL = row b). */
struct NPRSResult ECCR_AMD_reconstruct_batch_ws(
    unsigned long n_validators, const uint8_t *d_shards, unsigned long shard_len,
    unsigned long shard_stride, const uint8_t *d_present, const uint16_t *d_err_log,
    const uint32_t *d_pattern, unsigned long batch, uint8_t *d_out, unsigned long out_stride,
    void *d_workspace, unsigned long workspace_bytes, void *stream);

/* ---- shared erasure patterns ------------------------
 * d_pattern [batch] (uint32): payload b's erasure pattern is row d_pattern[b]
 * of d_present / d_err_log (rows may be shared by any number of payloads;
 * NULL = row b).  The usual case: the same validators missing for every block,
 * i.e. ONE present row and ONE locator for the whole batch. */

/* d_pattern[b] = a row whose pattern (present flags of positions < n_validators)
 * equals payload b's and which is its own leader (d_pattern[l] == l), or b
 * itself; normally the smallest such index (a 64-bit hash collision between
 * different patterns only costs the sharing: each row then leads itself).
 * batch < 2^31 (else BAD_PAYLOAD, nothing launched). */
struct NPRSResult ECCR_AMD_dedup_patterns(unsigned long n_validators, const uint8_t *d_present,
                                          unsigned long batch, uint32_t *d_pattern, void *stream);

/* Locators of the rows b with d_pattern[b] == b only (the other rows of
 * d_err_log are left untouched; d_pattern NULL: every row). */
struct NPRSResult ECCR_AMD_error_locator_patterns(unsigned long n_validators,
                                                  const uint8_t *d_present,
                                                  const uint32_t *d_pattern, unsigned long batch,
                                                  uint16_t *d_err_log, void *stream);

/* ECCR_AMD_reconstruct_batch with payload b's pattern = row d_pattern[b]. */
struct NPRSResult ECCR_AMD_reconstruct_batch_patterns(
    unsigned long n_validators, const uint8_t *d_shards, unsigned long shard_len,
    unsigned long shard_stride, const uint8_t *d_present, const uint16_t *d_err_log,
    const uint32_t *d_pattern, unsigned long batch, uint8_t *d_out, unsigned long out_stride,
    void *stream);

/* Hits / misses of the per-device locator cache of ECCR_reconstruct (the
 * locator of a pattern is computed once and reused while it is among the 64
 * most recent patterns). */
struct NPRSResult ECCR_AMD_locator_cache_stats(unsigned long *hits, unsigned long *misses);

/* Device-resident batch reconstruct_from_systematic (shards 0..k-1 of each
 * payload, same [batch][n_validators][shard_stride] layout). */
struct NPRSResult ECCR_AMD_systematic_batch(unsigned long n_validators, const uint8_t *d_shards,
                                            unsigned long shard_len, unsigned long shard_stride,
                                            unsigned long batch, uint8_t *d_out,
                                            unsigned long out_stride, void *stream);

/* ---- host-resident batches --------------------------
 * Stream a host batch through the device in chunks of `chunk` payloads (0 =
 * automatic: ~16 MB over the link per chunk), three chunks in flight (H2D /
 * kernels / D2H overlap).  Synchronous:
 * returns when the output is in host memory.  Host buffers should come from
 * ECCR_AMD_host_alloc (pinned) for full PCIe rate. */
void *ECCR_AMD_host_alloc(unsigned long bytes);
void ECCR_AMD_host_free(void *ptr);

/* payloads [batch][payload_stride] -> shards [batch][n_validators][shard_stride] */
struct NPRSResult ECCR_AMD_encode_host_batch(unsigned long n_validators, const uint8_t *h_payloads,
                                             unsigned long payload_len,
                                             unsigned long payload_stride, unsigned long batch,
                                             uint8_t *h_shards, unsigned long shard_stride,
                                             unsigned long chunk);

/* `count` present shards per payload, compacted: h_shards [batch][count][shard_stride]
 * with their validator indices h_index [batch][count] (a repeated index counts
 * once and must carry identical bytes) -> h_out [batch][out_stride >= shard_len*k].
 * Payloads with the same set of indices share one erasure locator per chunk.
 * Errors as ECCR_reconstruct: CHUNK_INDEX_OUT_OF_BOUNDS, NOT_ENOUGH_CHUNKS (< k
 * distinct), UNEVEN_LENGTH. */
struct NPRSResult ECCR_AMD_reconstruct_host_batch(unsigned long n_validators,
                                                  const uint8_t *h_shards, unsigned long shard_len,
                                                  unsigned long shard_stride,
                                                  const uint16_t *h_index, unsigned long count,
                                                  unsigned long batch, uint8_t *h_out,
                                                  unsigned long out_stride, unsigned long chunk);

/* Cap on one scratch allocation in bytes (per device or per stream; 0 = no
 * cap, the default).  A call whose shape needs more fails with UNKNOWN_CODE_PARAM
 * (encode) / UNKNOWN_RECONSTRUCTION (reconstruct) exactly as when hipMalloc
 * runs out of memory; nothing is launched.  Applies to the per-call C ABI
 * and the device-batch calls; the host-batch pipeline's slots own their
 * (chunk-sized) scratch and are not capped.  For memory-constrained
 * deployments and the failure-path tests. */
void ECCR_AMD_set_scratch_limit(unsigned long bytes);

/* Frees the device scratch the plain batch calls keep for `stream` on the
 * current device (after synchronising `stream`); call it before destroying a
 * stream that issued batch calls.  Returns 1 if a buffer was kept, else 0. */
int ECCR_AMD_release_stream_scratch(void *stream);

/* Last error message of the calling thread ("" if none). */
const char *ECCR_AMD_last_error(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ERASURE_CODING_EC_AMD_H_ */
