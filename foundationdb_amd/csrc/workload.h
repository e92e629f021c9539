/*
 * workload.h -- deterministic synthetic Resolver batches.
 *
 * Not part of the drop-in boundary: used by bench.py and the tests to produce
 * the same batches on any host.  Batches come out in the fdbcs_batch_view
 * layout of include/fdbcs.h.
 *
 * Configs (BASELINE.json "configs"):
 *   1  skipListTest-shaped (fdbserver/SkipList.cpp:1412-1486): 2,500 txns,
 *      1 read + 1 write, key = 12 x '.' + BE32(U[0, 2e7)), range [k, k+1+U[0,10]),
 *      snapshot = i, now = i + 50, newOldest = i.
 *   2  5,000 txns, 5 reads (80 % point [k, k\0), 20 % [k, k+U[1,16]] as a
 *      128-bit big-endian integer) + 2 point writes, uniform 16-byte keys.
 *   3  as 2 with key = BE64(r * 0x9E3779B97F4A7C15) || "zzzzzzzz",
 *      r ~ Zipf(0.99) over 1e6 ranks.
 *   4  68-100-byte keys BE64(tenant<16) || 56-byte path || U[4,36] random
 *      bytes; 4 point reads + 1 wide read covering a log-uniform 1e-3..1e-1
 *      fraction of the tenant's key space; 2 point writes.
 *   5  as 2 with 1,000,000 txns (snapshots now - U[1e4, 2e5]).
 *   50 config-5 preload: 1,000,000 blind point writes, now = 1e5 * (i + 1),
 *      newOldest = 0.
 * Versions (configs 2-5): now_i = 1e7 + i * 1e4, newOldest = now - 5e6
 * (MAX_WRITE_TRANSACTION_LIFE_VERSIONS, fdbserver/Knobs.cpp:34), snapshot =
 * now - U[1e4, 2e5]; 0.1 % of txns get now - 5e6 - 2e4 (tooOld next batch).
 * RNG: xoshiro256** seeded by splitmix64(0x5EED0000 + config*1000 + i), one
 * stream per 1,024-transaction chunk.
 */
#ifndef FDBCS_WORKLOAD_H
#define FDBCS_WORKLOAD_H
#include <stdint.h>
#include "../../include/fdbcs.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fdbwl fdbwl;

/* txns = 0 selects the config's default batch size. threads = 0: all cores. */
fdbwl* fdbwl_create(int32_t config, int32_t txns, int32_t threads);
void   fdbwl_destroy(fdbwl* g);

/* Generates batch `index`.  *view points into generator-owned host memory that
 * stays valid until the next call on g. */
int    fdbwl_generate(fdbwl* g, int64_t index, fdbcs_batch_view* view, int64_t* now, int64_t* new_oldest);

/* ---- bench drivers (call the C ABI of libfdbcs.so, which must be loaded
 * with RTLD_GLOBAL first: this library leaves the fdbcs_* symbols to it) ---- */

/* Batches [first, first + n) generated ahead of time and kept in the
 * Resolver's form: per transaction its read / write KeyRangeRefs into one key
 * arena and its read_snapshot (CommitTransactionRef, fdbclient/
 * CommitTransaction.h:89-100), plus (now, newOldest). */
typedef struct fdbwl_run fdbwl_run;
fdbwl_run* fdbwl_run_prepare(fdbwl* g, int64_t first, int32_t n);
void       fdbwl_run_destroy(fdbwl_run* r);
/* As fdbwl_run_prepare, each batch reduced to rank `resolver`'s input under
 * the exact sharded protocol B (fdbcs_split_batch_keep_all: every
 * transaction, only the ranges on the rank's keys), generated and split
 * before the clock as the proxy splits before the resolver receives. */
fdbwl_run* fdbwl_run_prepare_split(fdbwl* g, int64_t first, int32_t n, int32_t nres, const uint8_t* bound_bytes,
                                   const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver);
/* Transactions per batch (every prepared batch has the same count). */
int32_t    fdbwl_run_txns(const fdbwl_run* r);
/* Key bytes of prepared batch i (every begin and end key of its ranges). */
uint64_t   fdbwl_run_key_bytes(const fdbwl_run* r, int32_t i);

/* The Resolver's loop (Resolver.actor.cpp:140-153) over the prepared batches:
 * per batch ConflictBatch (fdbcs_batch_begin), T x addTransaction
 * (fdbcs_batch_add), detectConflicts (fdbcs_batch_detect).  batch_us[i] = the
 * wall time of batch i's window, add_us[i] its addTransaction part (both
 * optional); verdicts (optional) = n x T bytes. */
int fdbwl_run_resolver(fdbwl_run* r, fdbcs* cs, double* batch_us, double* add_us, uint8_t* verdicts);
/* The same loop with resolverCount > 1 (Resolver.actor.cpp:146-151): after
 * each detectConflicts, fdbcs_sample_add_batch(sample, cs, NULL,
 * offset_per_key, expire0 + i * expire_step, NULL) inside the batch's window
 * (sample: an fdbcs_sample, attached to cs or not). */
int fdbwl_run_resolver_sampled(fdbwl_run* r, fdbcs* cs, void* sample, int64_t offset_per_key, double expire0,
                               double expire_step, double* batch_us, double* add_us, uint8_t* verdicts);
/* The same loop on one rank of an exact sharded resolver
 * (fdbcs_sharded_batch_begin / _add / _detect). */
int fdbwl_run_resolver_sharded(fdbwl_run* r, fdbcs_sharded* sh, double* batch_us, double* add_us,
                               uint8_t* verdicts);

/* Grow a conflict set's history through n generated batches [first, first+n)
 * (fdbcs_batch_submit_packed / fdbcs_batch_wait, generation of batch i+1
 * overlapping batch i): the bench's steady-state prefill. */
// Config 4's wide reads end at the S-th boundary after their begin in the
// current history; fn answers a batch of such queries (the signature of
// fdbcs_nth_after: fdbwl_succ_engine with ctx = an fdbcs*, or the oracle's).
typedef int (*fdbwl_succ_fn)(void* ctx, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off,
                             const uint32_t* key_len, const int64_t* steps, uint8_t* out, uint32_t out_stride,
                             int32_t* out_len);
void fdbwl_set_successor(fdbwl* g, fdbwl_succ_fn fn, void* ctx);
int fdbwl_succ_engine(void* cs, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off, const uint32_t* key_len,
                      const int64_t* steps, uint8_t* out, uint32_t out_stride, int32_t* out_len);
// (measurement) the adds of fdbwl_run_resolver alone, no detect
int fdbwl_run_adds(fdbwl_run* r, fdbcs* cs, double* add_us);
int fdbwl_prefill(fdbwl* g, fdbcs* cs, int64_t first, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
