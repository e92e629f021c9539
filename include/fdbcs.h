/*
 * fdbcs.h -- C ABI of the MI355X-native FoundationDB Resolver conflict set.
 *
 * This is the drop-in boundary for the Resolver's conflict-detection engine.
 * In the reference that engine is fdbserver/SkipList.cpp behind
 * fdbserver/ConflictSet.h; its only production caller is
 * fdbserver/Resolver.actor.cpp:47,51,140-166.  Every entry point below says
 * which reference interface it replaces.  The C++ drop-in TU
 * (foundationdb_amd/shim/ConflictSetShim.cpp) maps ConflictSet.h onto these
 * calls 1:1; see INTEGRATION.md.
 *
 * Conventions
 *   - Plain pointers and sizes only; no C++ or torch types.
 *   - Every function returning int returns 0 on success and a negative
 *     FDBCS_E* code on failure (the reference ASSERTs -> internal_error,
 *     flow/Error.h:86; the shim turns a nonzero status into that throw).
 *   - Calls on one fdbcs are strictly serialized, as in the reference
 *     (Resolver.actor.cpp:104-122: one network thread, batches in version
 *     order).  Different fdbcs objects are independent.
 *   - Keys are byte strings compared unsigned-lexicographically, a proper
 *     prefix first (SkipList.cpp:113-120).  Every range must satisfy
 *     begin < end (reference precondition); violating it
 *     returns FDBCS_E_RANGE.
 */
#ifndef FDBCS_H
#define FDBCS_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Verdict bytes: numeric values of ConflictBatch::TransactionCommitResult
 * (ConflictSet.h:36-40).  The proxy takes the min across resolvers
 * (MasterProxyServer.actor.cpp:566), so the order matters. */
#define FDBCS_CONFLICT  0
#define FDBCS_TOO_OLD   1
#define FDBCS_COMMITTED 2

/* Status codes. */
#define FDBCS_OK          0
#define FDBCS_E_HIP      -1   /* a HIP runtime call failed                    */
#define FDBCS_E_NOMEM    -2   /* device or host allocation failed             */
#define FDBCS_E_RANGE    -3   /* a range with begin >= end                     */
#define FDBCS_E_STATE    -4   /* call out of order (e.g. add without begin)    */
#define FDBCS_E_ARG      -5   /* bad argument (null pointer, negative count)   */
#define FDBCS_E_KEY      -6   /* key longer than FDBCS_MAX_KEY                 */
#define FDBCS_E_NODEV    -7   /* no HIP device / extension not usable          */
#define FDBCS_E_CAPACITY -8   /* an internal device capacity was exceeded      */

/* Longest key accepted: SYSTEM_KEY_SIZE_LIMIT (fdbclient/Knobs.cpp:58) plus
 * one byte for keyAfter() (fdbclient/FDBTypes.h:269-279). */
#define FDBCS_MAX_KEY 30001

typedef struct fdbcs fdbcs;

/* One conflict range [begin, end) -- KeyRangeRef (fdbclient/FDBTypes.h:161). */
typedef struct fdbcs_range {
    const uint8_t* begin;
    uint32_t       begin_len;
    const uint8_t* end;
    uint32_t       end_len;
} fdbcs_range;

/*
 * A whole batch in packed structure-of-arrays form.  All pointers are either
 * host pointers (fdbcs_batch_detect_packed) or device pointers
 * (fdbcs_detect_device).  Transaction t owns reads
 * [read_off[t], read_off[t+1]) and writes [write_off[t], write_off[t+1]).
 * Key slots: read r has begin slot 2r and end slot 2r+1; write w has begin
 * slot 2R+2w and end slot 2R+2w+1 (R = read_count).  Slot s is the byte
 * string key_bytes[key_off[s] .. key_off[s]+key_len[s]).
 * Every transaction is listed, including ones that will turn out tooOld: the
 * engine applies the tooOld rule itself (SkipList.cpp:985), so a staged batch
 * does not depend on the conflict set's state.
 */
typedef struct fdbcs_batch_view {
    int32_t         txn_count;      /* T */
    int32_t         read_count;     /* R */
    int32_t         write_count;    /* W */
    int32_t         reserved;
    const int64_t*  snapshot;       /* [T]   CommitTransactionRef::read_snapshot */
    const int32_t*  read_off;       /* [T+1] */
    const int32_t*  write_off;      /* [T+1] */
    const uint64_t* key_off;        /* [2R+2W] */
    const uint32_t* key_len;        /* [2R+2W] */
    const uint8_t*  key_bytes;
    uint64_t        key_bytes_len;
} fdbcs_batch_view;

/* Optional construction parameters (NULL = defaults). */
typedef struct fdbcs_config {
    int32_t  device;            /* HIP device ordinal, -1 = current            */
    int32_t  flags;             /* FDBCS_BORROW_* below (0 = copy every key)   */
    int64_t  max_history;       /* boundaries to pre-size for (0 = default)    */
    int64_t  max_batch_keys;    /* key slots per batch to pre-size (0 = grow)  */
    int64_t  tail_arena_bytes;  /* device bytes for keys > 17 B (0 = default)  */
} fdbcs_config;

/* fdbcs_config.flags: how fdbcs_batch_add holds the caller's keys.
 *   FDBCS_BORROW_ALWAYS: every per-transaction batch borrows the caller's
 *     range arrays and key bytes until fdbcs_batch_detect returns, as the
 *     reference's addTransaction keeps StringRefs into the request's arena
 *     (SkipList.cpp:993-1004); the add records the pointers only, and
 *     detectConflicts checks and packs the batch on host threads.
 *   FDBCS_BORROW_LARGE: borrow when the previous per-transaction batch had at
 *     least FDBCS_BORROW_MIN_TXNS transactions (config 5's 10^6-transaction
 *     batches), copy otherwise.
 * A borrowed batch refuses nothing at add time: a transaction the add would
 * refuse (FDBCS_E_KEY / FDBCS_E_RANGE) makes fdbcs_batch_detect return that
 * status with the history unchanged (the reference ASSERTs inside
 * detectConflicts, SkipList.cpp:1117, 1127), and fdbcs_batch_refused_txn
 * names the first such transaction. */
#define FDBCS_BORROW_ALWAYS 1
#define FDBCS_BORROW_LARGE  2
#define FDBCS_BORROW_MIN_TXNS 65536

/* ---- ConflictSet lifecycle ------------------------------------------------ */

/* newConflictSet() (ConflictSet.h:28, SkipList.cpp:956): empty history, every
 * key at version v0 (the reference always uses 0), oldestVersion 0,
 * removalKey "". */
int  fdbcs_create(fdbcs** out, int64_t v0, const fdbcs_config* cfg);

/* clearConflictSet(cs, v) (ConflictSet.h:29, SkipList.cpp:957-959): history
 * reset to "every key at version v"; oldestVersion and removalKey are kept. */
int  fdbcs_clear(fdbcs* cs, int64_t v);

/* Alias named by the north star; identical to fdbcs_clear. */
int  fdbcs_set_version(fdbcs* cs, int64_t v);

/* destroyConflictSet() (ConflictSet.h:30, SkipList.cpp:960-962). */
void fdbcs_destroy(fdbcs* cs);

/* ---- ConflictBatch ----------------------------------------------------------- */

/* ConflictBatch::ConflictBatch(cs) (ConflictSet.h:33, SkipList.cpp:964-967):
 * starts an empty batch on cs. */
int  fdbcs_batch_begin(fdbcs* cs);

/* ConflictBatch::addTransaction(tr) (ConflictSet.h:42, SkipList.cpp:979-1008).
 * Transaction index = call order within the batch.  The key bytes are
 * copied into pinned staging memory before this returns, so the caller's
 * arena may be released at once (stricter than the reference, which borrows
 * them until detectConflicts returns).  A range with begin >= end
 * (FDBCS_E_RANGE) or a key over FDBCS_MAX_KEY (FDBCS_E_KEY) refuses the
 * transaction: it is not added, and the batch goes on.  A borrowed batch
 * (fdbcs_config.flags, FDBCS_BORROW_*) records the pointers only: the range
 * arrays and key bytes must stay valid until fdbcs_batch_detect returns. */
int  fdbcs_batch_add(fdbcs* cs, int64_t read_snapshot,
                     const fdbcs_range* reads, int32_t nreads,
                     const fdbcs_range* writes, int32_t nwrites);

/* n transactions with no ranges, as n addTransaction calls with empty read
 * and write lists (such a transaction always commits: tooOld needs a read,
 * SkipList.cpp:985) -- one call for a run of them.  A protocol-B shard
 * (fdbcs_sharded_set_protocol) skips the transactions the proxy did not send
 * it, keeping the others at their global batch indices. */
int  fdbcs_batch_skip(fdbcs* cs, int32_t n);

/* ConflictBatch::detectConflicts(now, newOldestVersion, nonConflicting,
 * tooOld) (ConflictSet.h:43, SkipList.cpp:1163-1208), synchronous.
 * verdict[t] receives FDBCS_CONFLICT / FDBCS_TOO_OLD / FDBCS_COMMITTED for
 * each of the batch's T transactions (T = number of fdbcs_batch_add calls).
 * Ends the batch. */
int  fdbcs_batch_detect(fdbcs* cs, int64_t now, int64_t new_oldest, uint8_t* verdict);

/* Number of transactions added to the current batch. */
int32_t fdbcs_batch_txn_count(const fdbcs* cs);

/* A borrowed batch that fdbcs_batch_detect refused: the index of its first
 * transaction with a range the add would have refused; -1 otherwise (no
 * reference counterpart: see FDBCS_BORROW_ALWAYS). */
int64_t fdbcs_batch_refused_txn(const fdbcs* cs);

/* Whole-batch variants of addTransaction x T + detectConflicts.
 *   _packed: host-resident batch view; copied H2D through pinned staging.
 *   _device: batch view whose arrays already live in device memory; verdict
 *            is a device pointer of T bytes.  If sync != 0 the call returns
 *            after the work completes, else it returns after enqueueing on the
 *            conflict set's stream (the next call orders behind it). */
int  fdbcs_batch_detect_packed(fdbcs* cs, const fdbcs_batch_view* host_batch,
                               int64_t now, int64_t new_oldest, uint8_t* verdict);
int  fdbcs_detect_device(fdbcs* cs, const fdbcs_batch_view* dev_batch,
                         int64_t now, int64_t new_oldest, uint8_t* dev_verdict,
                         int sync);

/* Pipelined host batches (batch ingest with overlapped
 * H2D).  The Resolver receives batches in version order while the previous one
 * is being resolved (Resolver.actor.cpp:104-122); submitting batch k+1 packs
 * it into a pinned staging slot and starts its host-to-device copy on a copy
 * stream while batch k's kernels run.  At most two batches are in flight;
 * fdbcs_batch_wait returns the oldest one's T verdict bytes (as
 * fdbcs_batch_detect_packed).  Results equal the synchronous calls'. */
int  fdbcs_batch_submit_packed(fdbcs* cs, const fdbcs_batch_view* host_batch, int64_t now, int64_t new_oldest);
int  fdbcs_batch_wait(fdbcs* cs, uint8_t* verdict);

/* ---- Key-range resolvers: the proxy side of multi-resolver scale-out ------------ */

/* ResolutionRequestBuilder::addTransaction (MasterProxyServer.actor.cpp:267-307)
 * for a static key -> resolver map of nres resolvers: resolver g owns keys in
 * [bound[g-1], bound[g]) with bound[-1] = "" and bound[nres-1] = +infinity;
 * the nres-1 bounds (strictly ascending) are bound_bytes[bound_off[i] ..
 * + bound_len[i]).  Writes into *out the sub-batch resolver `resolver`
 * receives: every transaction with at least one read or write range
 * intersecting its keys, in batch order, carrying all such ranges unclipped
 * and its read_snapshot; txn_index[i] = the sub-batch transaction's index in
 * the input.  The output arrays are caller-provided with the input's sizes
 * (T, T+1, T+1, 2R+2W, 2R+2W, T); out->key_bytes aliases in->key_bytes.
 * Host memory only. */
int  fdbcs_split_batch(const fdbcs_batch_view* in, int32_t nres, const uint8_t* bound_bytes,
                       const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver,
                       fdbcs_batch_view* out, int64_t* snapshot, int32_t* read_off, int32_t* write_off,
                       uint64_t* key_off, uint32_t* key_len, int32_t* txn_index);

/* As fdbcs_split_batch, but every transaction of the input stays in the
 * sub-batch (txn_index is the identity), with only the ranges intersecting
 * the resolver's keys -- plus the writes ending exactly at its first key,
 * whose end node it holds: the per-shard input of the exact sharded
 * protocol B, which keeps batch transaction indices global. */
int  fdbcs_split_batch_keep_all(const fdbcs_batch_view* in, int32_t nres, const uint8_t* bound_bytes,
                                const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver,
                                fdbcs_batch_view* out, int64_t* snapshot, int32_t* read_off, int32_t* write_off,
                                uint64_t* key_off, uint32_t* key_len, int32_t* txn_index);

/* The resolver owning key (keyResolvers lookup), or a negative status. */
int32_t fdbcs_key_owner(int32_t nres, const uint8_t* bound_bytes, const uint64_t* bound_off,
                        const uint32_t* bound_len, const uint8_t* key, uint32_t key_len);

/* The proxy's verdict combine (MasterProxyServer.actor.cpp:558-569), one
 * resolver's share: dev_global[dev_index[i]] = dev_sub[i] for i < n, on cs's
 * stream (NULL cs: the null stream).  dev_global starts as T bytes of
 * FDBCS_COMMITTED; the element-wise MIN over all resolvers' arrays (an RCCL
 * MIN all-reduce when the resolvers are GPUs) is the combined verdict. */
int  fdbcs_scatter_verdicts(fdbcs* cs, const uint8_t* dev_sub, const int32_t* dev_index, int32_t n,
                            uint8_t* dev_global);

/* ---- Exact sharded mode: one resolver over G GPUs (SURVEY.md §8e protocols A, B) ---- */

/* The north star's node layout: GPU g holds the history of the keys in
 * [lo, hi) (has_lo / has_hi == 0: unbounded), every GPU receives the whole
 * batch, and the host exchanges between the phases below.  The result equals
 * one ConflictSet's (a single Resolver, Resolver.actor.cpp:140-153) exactly.
 * A shard's header version (fdbcs_header_version) is its carry-in: the
 * version of the last boundary below lo anywhere, or the global v0. */
int  fdbcs_set_shard(fdbcs* cs, const uint8_t* lo, uint32_t lo_len, int has_lo,
                     const uint8_t* hi, uint32_t hi_len, int has_hi);

/* Phase 1 (steps 1-2): ingest, endpoint sort, intra-batch overlaps, and the
 * history check of every read clipped to the shard.  carry_in: the version of
 * the last boundary below lo after the previous batch's merge (its
 * compaction can change that only between versions below oldestVersion,
 * which no checked read can tell apart).  dev_hist receives T flag bytes
 * (2: tooOld -- SkipList.cpp:985 -- 1: the transaction conflicts with this
 * shard's history, 0: neither); the host MAX-reduces them over the shards
 * (RCCL all-reduce).  Protocol B: the batch holds every transaction of the
 * global batch but only the ranges intersecting [lo, hi)
 * (fdbcs_split_batch_keep_all); a transaction with no read here reports 0,
 * and the shard that holds one of its reads reports the tooOld flag. */
int  fdbcs_shard_check(fdbcs* cs, const fdbcs_batch_view* dev_batch, int64_t now,
                       int64_t new_oldest, int64_t carry_in, uint8_t* dev_hist);

/* Phase 2 (steps 4-5): the decision from the reduced flags (identical on
 * every shard, verdicts to dev_verdict), the combine, and the shard's part of
 * the merge.  carry_in: the exact carry-in after the previous batch's
 * compaction (end nodes created with no boundary below them in the shard
 * take it).  removal_key / removal_key_len >= 0: the removalKey the previous
 * batch's compaction produced (-1: unchanged).  info[0] = boundaries H,
 * [1] = index of the shard's first boundary >= removalKey when a compaction
 * follows (else -1), [2] = version of its last boundary (INT64_MIN: none),
 * [3] = combined write ranges whose begin lies in [lo, hi) (their sum over
 * the shards is |combinedWriteConflictRanges|, the compaction budget's
 * len(C), SkipList.cpp:1198-1206).  When new_oldest > oldestVersion,
 * fdbcs_shard_compact must follow.  Protocol B: fdbcs_shard_set_edges
 * first. */
int  fdbcs_shard_apply(fdbcs* cs, const fdbcs_batch_view* dev_batch, int64_t now, int64_t new_oldest,
                       int64_t carry_in, const uint8_t* removal_key, int32_t removal_key_len,
                       const uint8_t* dev_hist, uint8_t* dev_verdict, int64_t* info);

/* Phase 3 (step 6): removeBefore over this shard's part [a, b) of the global
 * window (local indices).  keep_first: a is the window's first node (never
 * removed); prev_version: the version of the node before local index 0 (the
 * previous non-empty shard's last).  key_index >= 0: this shard holds the
 * window's end -- the key there (the new removalKey) is read before the
 * compaction into key_buf (key_cap bytes).  info[0] = H, info[1] = last
 * version, info[2] = the key's length (-1: none read). */
int  fdbcs_shard_compact(fdbcs* cs, int64_t a, int64_t b, int keep_first, int64_t prev_version,
                         int64_t new_oldest, int64_t key_index, uint8_t* key_buf, int32_t key_cap,
                         int64_t* info);

/* Protocol B (for batches too large to sort on every GPU):
 * each shard receives only the ranges intersecting its keys, so the endpoint
 * sort, the overlap search and the history check are all shard-local.  Every
 * intra-batch overlap (read r of t, write w of u) has a non-empty
 * intersection inside some shard, where both ranges are present, so the union
 * of the shards' edge lists is the whole batch's.  sparse_edges != 0 makes
 * this shard keep its overlap pairs undeduplicated for export (before the
 * first batch).  Per batch: fdbcs_shard_check, then fdbcs_shard_edge_count /
 * fdbcs_shard_get_edges (the pairs (reader t, earlier writer u) in batch
 * transaction indices, into caller device memory), an all-gather of the
 * lists, fdbcs_shard_set_edges with their concatenation, fdbcs_shard_apply
 * (the ordered decision over the global edges -- identical on every shard --
 * then this shard's combine and merge). */
int     fdbcs_shard_set_protocol(fdbcs* cs, int sparse_edges);
int64_t fdbcs_shard_edge_count(fdbcs* cs);
int     fdbcs_shard_get_edges(fdbcs* cs, int32_t* dev_et, int32_t* dev_eu, int64_t n);
int     fdbcs_shard_set_edges(fdbcs* cs, const int32_t* dev_et, const int32_t* dev_eu, int64_t n);

/* ---- Introspection (tests, bench, checkpoint) --------------------------------- */

/* Number of boundaries in the history (skip-list nodes other than the header). */
int64_t fdbcs_history_size(fdbcs* cs);
/* Header version v0 and oldestVersion (ConflictSet::oldestVersion). */
int64_t fdbcs_header_version(const fdbcs* cs);
int64_t fdbcs_oldest_version(const fdbcs* cs);

/* Copies the history in key order: versions[i], key_len[i], key_off[i] (into
 * key_bytes).  Capacities are in elements / bytes; returns the number of
 * boundaries written or a negative status (FDBCS_E_CAPACITY if too small). */
int64_t fdbcs_dump_history(fdbcs* cs, int64_t cap, int64_t* versions, uint32_t* key_len,
                           uint64_t* key_off, uint8_t* key_bytes, uint64_t key_bytes_cap);
/* Replaces the history with the given sorted, distinct boundaries (v0, oldest
 * and removalKey are set from the arguments).  For tests and warm starts. */
int  fdbcs_load_history(fdbcs* cs, int64_t n, const int64_t* versions, const uint32_t* key_len,
                        const uint64_t* key_off, const uint8_t* key_bytes,
                        int64_t v0, int64_t oldest, const uint8_t* removal_key,
                        uint32_t removal_key_len);
/* ConflictSet::removalKey: copies up to cap bytes, returns the full length. */
int32_t fdbcs_removal_key(fdbcs* cs, uint8_t* buf, int32_t cap);

/* Per-stage device time of the last batch in microseconds, in the order of
 * the reference's PerfDoubleCounters (SkipList.cpp:91-111): [0] encode/sort
 * (D.Sort), [1] history read check (D.CheckRead), [2] intra-batch
 * (D.CheckIntraBatch), [3] combine (D.Combine), [4] merge (D.MergeWrite),
 * [5] compaction (D.RemoveBefore), [6] whole batch.  Only filled when stage
 * timing is enabled. Returns the number of entries written. */
int  fdbcs_enable_stage_timing(fdbcs* cs, int on);
int  fdbcs_stage_times(fdbcs* cs, double* out_us, int cap);

/* Shape and outcome of the last synchronized batch (bench byte models):
 * [0] T  [1] R  [2] W  [3] combined write ranges  [4] history pages the merge
 * rewrote  [5] directory entries  [6] history boundaries  [7] compaction
 * window pages  [8] boundaries surviving in them  [9] transactions with
 * intra-batch sources  [10] decision rounds  [11] 1: a sort bucket
 * overflowed and the batch's endpoints were bucketed again by splitters from
 * its own sample  [12] largest sort bucket above 128 records (0: none)
 * [13] tail arena bytes (both halves)  [14] bytes used in its current half
 * [15] current half (flips when a compaction sweep freed the other)
 * [16] per-transaction batches ingested live (during their adds) so far
 * [17] live batches cancelled on the way (outgrew the live capacities, or
 * another call needed the stream) and ingested whole at detect  [18] of
 * those, batches whose live kernel gave up waiting for the adds (its
 * timeout, FDBCS_LIVE_TIMEOUT_US, default 8 s).
 * Returns the count written. */
#define FDBCS_STATS 19
int  fdbcs_batch_stats(fdbcs* cs, int64_t* out, int cap);

/* Profiling builds only (-DFDBCS_PHASES): the 100 MHz device timestamps the
 * kernels recorded at their phase boundaries during the last synchronized
 * batch.  Returns the number of entries written (0 in normal builds). */
int  fdbcs_debug_phases(fdbcs* cs, int64_t* out, int cap);

/* Test hook: the searches' long-prefix skips of the current history
 * (DESIGN.md §4 "Long shared prefixes"): [0] directory windows (16 entries,
 * level 0) with a skip, [1] live pages with a skip (Pool::pskip > 0), [2]
 * live pages waiting for k_page_px (< 0).  Synchronizes.  Returns the count
 * written. */
int  fdbcs_debug_prefix_skips(fdbcs* cs, int64_t* out, int cap);

/* The HIP stream the conflict set enqueues on (as void*), for callers that
 * want to time or order around it. */
void* fdbcs_stream(fdbcs* cs);

/* Device view of the batch most recently resolved through a host path
 * (fdbcs_batch_detect / fdbcs_batch_detect_packed): its arrays stay valid in
 * device memory until the next batch is staged.  FDBCS_E_STATE when there is
 * none (nothing resolved yet, or a pipelined submit since). */
int  fdbcs_last_device_batch(fdbcs* cs, fdbcs_batch_view* out);

/* ---- Resolver load metrics ------------------------------------ */

/* The Resolver's iopsSample: TransientStorageMetricSample
 * (fdbserver/StorageMetrics.actor.h:98-182) constructed with
 * KEY_BYTES_PER_SAMPLE (fdbserver/Knobs.cpp:269, 2e4) units per sample,
 * Resolver.actor.cpp:47,65.  `seed` fixes the sample's draws (the reference
 * uses the unseeded g_random; see foundationdb_amd/csrc/load_metrics.hip). */
typedef struct fdbcs_sample fdbcs_sample;
int  fdbcs_sample_create(fdbcs_sample** out, int64_t units_per_sample, uint64_t seed);
void fdbcs_sample_destroy(fdbcs_sample* s);

/* Resolver.actor.cpp:146-151 for one whole batch: addAndExpire(begin,
 * offset_per_key + |begin|, expiration) for every write then every read range
 * of each transaction in batch order (offset_per_key = SAMPLE_OFFSET_PER_KEY,
 * Knobs.cpp:278, 100; expiration = now() + SAMPLE_EXPIRATION_TIME).  The roll
 * and the gather of the sampled keys run on the device, over dev_batch (a
 * device-resident batch view; NULL = fdbcs_last_device_batch(cs)), on cs's
 * stream; synchronous.  *out_sampled (optional) = keys sampled.
 * With the sample attached to cs (fdbcs_sample_attach) and dev_batch NULL
 * after a per-transaction batch (fdbcs_batch_detect), the roll was already
 * done by that batch's ingest on the device, and its entries came back with
 * the verdicts: the call only inserts them (no launch, no wait). */
int  fdbcs_sample_add_batch(fdbcs_sample* s, fdbcs* cs, const fdbcs_batch_view* dev_batch,
                            int64_t offset_per_key, double expiration, int64_t* out_sampled);

/* Attach the sample to cs (NULL: detach): from the next fdbcs_batch_detect
 * on, the per-transaction ingest rolls every range for this sample as it
 * encodes it (Resolver.actor.cpp:146-151, with this offset_per_key), writing
 * the sampled entries and begin keys to pinned host memory; the following
 * fdbcs_sample_add_batch(s, cs, NULL, offset_per_key, ...) consumes them.  A
 * batch the caller does not add (resolverCount <= 1) costs its draws nothing:
 * the draw counter advances only when a batch enters the sample.  One sample
 * per conflict set; destroying either detaches them. */
int  fdbcs_sample_attach(fdbcs_sample* s, fdbcs* cs, int64_t offset_per_key);

/* IndexedSet::addMetric on the sample without the roll or the queue
 * (flow/IndexedSet.h:587-598; StorageMetrics.actor.h's own test inserts this
 * way, :81-93).  An entry whose metric reaches 0 is erased.  A delta that
 * would leave the entry's metric below 0 is refused (FDBCS_E_ARG): the
 * Resolver's amounts are positive and expire back to 0, and the sample's
 * prefix-sum index assumes nondecreasing prefixes. */
int  fdbcs_sample_add_metric(fdbcs_sample* s, const uint8_t* key, uint32_t len, int64_t metric);

/* TransientStorageMetricSample::poll() (StorageMetrics.actor.h:150-164):
 * apply every queued expiry with expiration <= now
 * (Resolver.actor.cpp:286-289, every SAMPLE_POLL_TIME). */
int  fdbcs_sample_poll(fdbcs_sample* s, double now);

/* Threading of the queries below: they take a const handle, but each first
 * inserts the batches an attached engine rolled and fdbcs_sample_add_batch
 * queued (in batch order, so nothing observable moves) -- they MUTATE the
 * sample.  Like every other call on a sample, they are not thread-safe: one
 * thread at a time per sample, queries included (the Resolver's actor runs
 * them on its one network thread, Resolver.actor.cpp:276-289). */
/* getEstimate(KeyRangeRef(b, e)) (StorageMetrics.actor.h:35-37): the sum of
 * the sampled metrics of keys in [b, e).  ResolutionMetricsRequest answers
 * getEstimate(allKeys) (Resolver.actor.cpp:276-277). */
int64_t fdbcs_sample_estimate(const fdbcs_sample* s, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el);

/* splitEstimate(KeyRangeRef(b, e), offset, front) (StorageMetrics.actor.h:38-73;
 * ResolutionSplitRequest, Resolver.actor.cpp:279-283).  Writes the split key
 * into out (cap bytes) and returns its length, or a negative status. */
int32_t fdbcs_sample_split(const fdbcs_sample* s, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el,
                           int64_t offset, int front, uint8_t* out, uint32_t cap);

/* Sampled keys held, queued expiries, and entry i (ascending key order):
 * key bytes into out (length returned), its metric into *metric. */
int64_t fdbcs_sample_size(const fdbcs_sample* s);
int64_t fdbcs_sample_queue_size(const fdbcs_sample* s);
int32_t fdbcs_sample_entry(const fdbcs_sample* s, int64_t i, uint8_t* out, uint32_t cap, int64_t* metric);

/* History query (bench / test support): for each of
 * n keys, the key of the boundary `steps[i]` positions after the first
 * boundary >= key i, into out + i * out_stride (out_len[i] = its length, or -1
 * past the last boundary; a key longer than out_stride is not copied).
 * Synchronous; sees every batch already resolved. */
int  fdbcs_nth_after(fdbcs* cs, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off,
                     const uint32_t* key_len, const int64_t* steps, uint8_t* out, uint32_t out_stride,
                     int32_t* out_len);

/* Human-readable message for a status code. */
const char* fdbcs_strerror(int status);

/* Library build identification (git-independent): "fdbcs gfx950 <version>". */
const char* fdbcs_version(void);

/* ---- One Resolver over G GPUs (SURVEY.md §8e protocols A and B) ---------
 * Replaces the proxy's split over G resolvers (MasterProxyServer.actor.cpp:
 * 242-320) with one exact resolver: the verdicts, the concatenated history,
 * removalKey and oldestVersion equal one ConflictSet's
 * (ConflictSet.h:27-60) bit for bit.  One process (rank) per GPU; rank g
 * holds the keys [bound[g-1], bound[g]) and receives every transaction.
 * Per batch two exchanges run on the engine's stream (RCCL all-reduce MAX of
 * the abort flags + per-shard slots, all-gather of per-shard counts); the
 * carry-ins, the compaction plan and removalKey's owner are computed on the
 * device; the host waits once, for the verdicts. */
typedef struct fdbcs_sharded fdbcs_sharded;

#define FDBCS_COMM_ID_BYTES 128

/* Host-memory collectives over the ranks (tests: torch.distributed gloo).
 * Each returns 0 on success. */
typedef struct fdbcs_comm_ops {
    void* ctx;
    /* element-wise MAX over ranks of n bytes, in place */
    int (*allreduce_max_u8)(void* ctx, uint8_t* buf, uint64_t n);
    /* rank r's n bytes land at recv[r * n .. (r + 1) * n) on every rank */
    int (*allgather_u8)(void* ctx, const uint8_t* send, uint8_t* recv, uint64_t n);
} fdbcs_comm_ops;

/* An RCCL unique id (rank 0 makes it; the caller hands it to every rank). */
int  fdbcs_comm_unique_id(uint8_t* id /* FDBCS_COMM_ID_BYTES */);

/* newConflictSet() for rank `rank` of `world` (SkipList.cpp:956).  bounds:
 * world - 1 increasing split keys (key i at bound_bytes + bound_off[i],
 * bound_len[i] bytes).  Exactly one of comm_id (RCCL, one GPU per rank, the
 * device from cfg) or ops (host collectives) is given. */
int  fdbcs_sharded_create(fdbcs_sharded** out, int32_t rank, int32_t world, const uint8_t* bound_bytes,
                          const uint64_t* bound_off, const uint32_t* bound_len, int64_t v0,
                          const fdbcs_config* cfg, const uint8_t* comm_id, const fdbcs_comm_ops* ops);
/* comm_id and ops both NULL: the communicator is joined later, once every
 * rank's create has succeeded (a rank that fails here then never leaves the
 * others waiting inside ncclCommInitRank). */
int  fdbcs_sharded_comm_init(fdbcs_sharded* sh, const uint8_t* comm_id);
/* From any thread: ends this rank's in-flight RCCL collectives
 * (ncclCommAbort) so a batch whose peer failed returns an error instead of
 * waiting forever; every later call on sh fails.  Host collectives
 * (fdbcs_comm_ops) must be released by their owner. */
int  fdbcs_sharded_abort(fdbcs_sharded* sh);
void fdbcs_sharded_destroy(fdbcs_sharded* sh);
/* clearConflictSet (SkipList.cpp:957-959), on every rank. */
int  fdbcs_sharded_clear(fdbcs_sharded* sh, int64_t v);
/* ConflictBatch on the sharded set: the same calls as fdbcs_batch_*, on every
 * rank with the same transactions; every rank receives all T verdicts. */
int  fdbcs_sharded_batch_begin(fdbcs_sharded* sh);
int  fdbcs_sharded_batch_add(fdbcs_sharded* sh, int64_t read_snapshot, const fdbcs_range* reads, int32_t nreads,
                             const fdbcs_range* writes, int32_t nwrites);
int  fdbcs_sharded_batch_skip(fdbcs_sharded* sh, int32_t n);
int  fdbcs_sharded_batch_detect(fdbcs_sharded* sh, int64_t now, int64_t new_oldest, uint8_t* verdict);
/* A device-resident batch view (protocol A: every rank the whole batch;
 * protocol B: this rank's fdbcs_split_batch_keep_all share); host verdicts. */
int  fdbcs_sharded_detect_device(fdbcs_sharded* sh, const fdbcs_batch_view* dev_batch, int64_t now,
                                 int64_t new_oldest, uint8_t* verdict);

/* Protocol B (the bench's N > 1 default): each rank takes
 * only the ranges that intersect its keys (and the writes ending exactly at
 * its first key), so ingest, endpoint sort and overlap search stay
 * shard-local instead of growing with the whole batch.  Transactions keep
 * their global batch indices (a rank with none of a transaction's ranges
 * still counts it).  Exchange 1 also carries each rank's overlap-edge count;
 * one all-gather of a fixed capacity of edge pairs per rank follows with no
 * host read in between (a batch whose lists do not fit runs from exchange 1
 * again with a larger capacity; the capacity decays back once a window of
 * batches needed at most half of it), and every rank runs the identical
 * ordered decision over their union.  Flags: FDBCS_SHARD_PRESPLIT
 * = the caller's adds already carry only this rank's ranges (the proxy's
 * per-resolver split, fdbcs_split_batch_keep_all); without it
 * fdbcs_sharded_batch_add drops the others itself (after checking every
 * range, so all ranks refuse the same transactions).  A PRESPLIT caller must
 * have validated every range of each global transaction (begin < end, key
 * lengths) before splitting it: a rank sees only its share, so a
 * transaction refused on one rank and accepted on another would give the
 * ranks different transaction counts, and exchange 1 (sized by T) would
 * mismatch across ranks.  Between batches. */
#define FDBCS_PROTOCOL_A     0
#define FDBCS_PROTOCOL_B     1
#define FDBCS_SHARD_PRESPLIT 1
int  fdbcs_sharded_set_protocol(fdbcs_sharded* sh, int protocol, int flags);
/* Protocol B's edge exchange (no reference counterpart: instrumentation of
 * the sharded mode): [0] edge pairs per rank the all-gather carries now
 * [1] batches whose exchange was short and ran again [2] the last batch's
 * largest rank edge count [3] times the capacity decayed [4] the exchange
 * buffer's int32 elements.  Returns the count written. */
int  fdbcs_sharded_exchange_stats(const fdbcs_sharded* sh, int64_t* out, int cap);
/* This rank's engine: its part of the history (fdbcs_dump_history,
 * fdbcs_history_size); the owner's fdbcs_removal_key is removalKey. */
fdbcs* fdbcs_sharded_local(fdbcs_sharded* sh);
/* The rank holding removalKey (-1: removalKey is ""). */
int32_t fdbcs_sharded_removal_key_owner(fdbcs_sharded* sh);
int64_t fdbcs_sharded_header_version(const fdbcs_sharded* sh);

#ifdef __cplusplus
}
#endif

#endif /* FDBCS_H */
