// stage.h -- host staging of ConflictBatch::addTransaction (SkipList.cpp:979-1008)
// for the per-transaction path (fdbcs_batch_add / fdbcs_batch_detect).
//
// The Resolver calls addTransaction T times on one thread, then
// detectConflicts (Resolver.actor.cpp:140-153).  Each call checks its ranges
// and appends one record -- a StageHdr, the range lengths, the key bytes
// (kernels.h) -- to a pinned byte stream: the only host copy of the batch.
// Every `chunk` bytes the new part of the stream starts its H2D copy on a
// copy stream of its own, so most of the batch is on the device by the time
// detectConflicts is called -- while the previous batch's history update is
// still running on the conflict set's stream (copies queued behind it there
// held every batch up by ~90 us).  finish() appends the record offsets to the
// stream, sends the rest in one copy, makes the conflict set's stream wait for
// it, and k_unpack builds the batch view on the device.  One device buffer
// suffices: the previous batch's k_unpack (the only reader of the record
// bytes; the encoder copies key tails into the batch's own buffer) finished
// before its verdicts came back, i.e. before this batch's first add.
//
// (Measured and dropped: handing the record copies to helper threads during
// the adds -- the calling thread got slower, 185 -> 250-990 us per config-2
// batch -- and a parallel gather at detect by 8 host threads over borrowed
// ranges: 52-65 us for the gather, but the 1.5 MB H2D no longer overlapped
// the adds (~25 GB/s) and the caller's add loop slowed 3x while the helper
// threads lived, for no net gain.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "kernels.h"

namespace fdbcs_dev {

class HostPool;  // (stage.hip: the borrowed batches' packing threads)

class TxnStage {
   public:
    TxnStage() = default;
    ~TxnStage() { release(); }
    TxnStage(const TxnStage&) = delete;
    TxnStage& operator=(const TxnStage&) = delete;

    // stream: where k_unpack goes; copy: where the H2D copies go (event-joined
    // into stream); chunk: bytes per streamed copy
    int configure(hipStream_t stream, hipStream_t copy, uint64_t chunk);
    // free the buffers and forget the stream (before the owner destroys it)
    void release();

    // borrow: the adds record the caller's range arrays only, as the
    // reference's addTransaction keeps StringRefs into the caller's arena until
    // detectConflicts returns (SkipList.cpp:993-1004); finish() then checks and
    // packs the whole batch on host threads (pack_borrowed).  Large batches
    // (config 5: 10^6 transactions) no longer pack on the caller's one core.
    int begin(bool borrow = false);
    bool borrowing() const { return borrow_; }
    // a borrowed batch refused at finish(): the first transaction whose
    // ranges the add would have refused (-1: none)
    int64_t refused_at() const { return bad_txn_; }
    // this batch began live (begin_live): a refused one must have the live
    // kernel's partial work undone (the engine's k_live_reset)
    bool began_live() const { return began_live_; }
    // a live batch that borrows: helper threads pack it while the adds go on
    bool live_borrowed() const { return lb_; }
    // A borrowed batch that does not go live: helper threads pack it during
    // the adds and send it to the device as it grows (caps: as the live
    // capacities, for the helpers' buffers; a batch past them is packed at
    // finish instead)
    int begin_helpers(const LiveCaps& caps);
    // Live ingest: after begin(), make this batch live --
    // the stream, offsets and view sized for `caps`, the progress words reset
    // -- before the engine launches k_live_ingest over them.  The adds then
    // publish their progress instead of copying chunks; a batch that leaves
    // `caps` (or a buffer that must grow) is cancelled and ingested at
    // finish() as usual.
    int begin_live(const LiveCaps& caps);
    // The most stream bytes a live batch within `caps` can reach (records,
    // the padding of every publish and of the final word): the batch tail
    // buffers are sized by it before the live kernel writes them
    // (engine.hip live_begin), so detectConflicts never has to move them.
    uint64_t live_stream_bound(const LiveCaps& caps) const;
    // live batches whose kernel gave up (LiveTune::timeout_ticks) and that
    // finish() sent to the whole-stream ingest instead
    int64_t live_timeouts() const { return timeouts_; }
    // the live kernel's inputs (device pointers of the host-mapped buffers)
    const uint8_t* stream_dev() const { return pin_dev_; }
    uint64_t stream_cap() const { return cap_; }
    const uint64_t* toff_dev() const { return toff_dev_; }
    const uint64_t* prog_dev() const { return prog_dev_; }
    UnpackOut live_view() const { return lview_; }
    bool live_active() const { return live_ && !live_broken_; }
    // cancel a live batch (the kernel leaves; finish() ingests the whole stream)
    void live_cancel();
    // addTransaction: FDBCS_E_KEY / FDBCS_E_RANGE (begin >= end, SURVEY.md
    // §0.6) refuse the transaction, which is then not part of the batch.
    int add(int64_t snap, const fdbcs_range* reads, int32_t nr, const fdbcs_range* writes, int32_t nw);
    // n transactions without ranges (add(_, _, 0, _, 0) n times, one offset entry each)
    int skip(int32_t n);
    // Sends the rest; dv = the device batch view (valid until the next
    // begin()).  With `staged`, the next ingest builds dv's arrays itself
    // straight from the stream (*staged: where to find it); else k_unpack
    // builds them now (FDBCS_SEPARATE_UNPACK: always).  A live batch: the
    // final progress word instead (staged->live; dv over the host-mapped
    // stream and the live view layout).
    int finish(fdbcs_batch_view& dv, StagedBatch* staged = nullptr);
    int64_t txns() const { return T_; }
    int64_t reads() const { return R_; }
    int64_t writes() const { return W_; }
    uint64_t stream_bytes() const { return used_; }
    // the batch's key bytes (every begin and end key): more than the stream
    // holds when point ranges share their bytes; sizes the tail buffers
    uint64_t key_total() const { return K_; }
    bool open() const { return open_; }

   private:
    int grow(int64_t need_txns, uint64_t need_bytes);
    int grow_bar(int64_t need_txns, uint64_t need_bytes);
    void publish();
    bool pad_published();
    void live_check();

    void sync();
    static bool pull_rest();
    int pack_borrowed();
    void drop_pool();
    // Live borrowed batches (begin_live after begin(true)): the caller's adds
    // record pointers; helper threads of the pool take chunks of LB_CHUNK
    // transactions as they are added, check and pack them into the stream in
    // chunk order and publish them to the live kernel -- the copy and the
    // checks leave the caller's thread, and the device still encodes the
    // batch during the adds.
    struct LbShared;
    LbShared* lbs_ = nullptr;
    bool lb_ = false;
    bool lb_live_ = false;  // the helpers publish to the live kernel (else they copy)
    bool began_live_ = false;
    int start_helpers(bool live);
    void lb_work();
    void lb_abandon();  // stop the helpers; the batch goes on as a plain borrowed one
    HostPool* pool_ = nullptr;  // created at the first borrowed batch large enough to share
    struct BorrowRec {
        int64_t snap;
        const fdbcs_range* rd;
        const fdbcs_range* wr;
        int32_t nr, nw;
    };
    bool borrow_ = false;
    // the adds' records: written with non-temporal stores (a 10^6-transaction
    // batch's 32 MB would otherwise be read for ownership first: 3x slower)
    BorrowRec* brec_ = nullptr;
    int64_t brec_cap_ = 0;
    int grow_brec(int64_t need);
    int64_t bad_txn_ = -1;
    bool toff_in_stream_ = false;  // pack_borrowed wrote the record offsets after the records

    hipStream_t stream_ = nullptr;
    hipStream_t copy_ = nullptr;
    hipEvent_t copied_ = nullptr;
    uint64_t chunk_ = 512 << 10;
    uint64_t early_ = 128 << 10;       // FDBCS_STAGE_EARLY: bytes before the predicted end (0: off)
    uint64_t early_at_ = ~0ull;        // where this batch's extra chunk goes
    bool open_ = false;
    int64_t T_ = 0, R_ = 0, W_ = 0;
    uint64_t K_ = 0;
    // the record stream: pinned + device copy, same capacity
    uint8_t* pin_ = nullptr;
    uint8_t* pin_dev_ = nullptr;  // pin_ as the device sees it (mapped)
    uint8_t* dev_ = nullptr;
    bool chunk_sent_ = false;     // a chunk copy (and its event) since begin()
    uint64_t cap_ = 0;
    uint64_t used_ = 0, sent_ = 0;
    uint64_t* toff_ = nullptr;    // pinned, host-mapped [T]: record offsets (appended to the stream at finish)
    uint64_t* toff_dev_ = nullptr;
    bool pin_live_ = false, toff_live_ = false;  // the stream / offsets are coherent (live ingest can read them)
    // FDBCS_STAGE_BAR=1: the stream, offsets and progress words are device
    // memory the host writes through the large BAR (fine-grained, uncached
    // on the device): no chunk copies, the kernels read them from HBM
    // (configure(); slower adds, so off by default)
    bool bar_ = false;
    int64_t toff_cap_ = 0;
    uint8_t* view_ = nullptr;     // device: the unpacked arrays
    uint64_t view_cap_ = 0;
    // live ingest
    bool live_ = false;           // this batch began live ...
    bool live_broken_ = false;    // ... and was cancelled (finish() ingests it whole)
    LiveCaps lcaps_{};
    UnpackOut lview_{};           // the view's arrays in the live layout (sized by lcaps_)
    int64_t pub_every_ = 16;      // FDBCS_LIVE_PUB: transactions per progress word
    int64_t timeouts_ = 0;
    int64_t next_pub_ = 0;
    // host-mapped progress: [0] published bytes << 20 | published T (one
    // word; LV_FINAL_BIT once the batch is whole), [1] final stream bytes,
    // [2] state (LV_RUNNING / LV_FINAL / LV_CANCEL), [3..5] final T, R, W,
    // [6] set by the live kernel's poller when it gave up (timeout)
    uint64_t* prog_ = nullptr;
    uint64_t* prog_dev_ = nullptr;
};

}  // namespace fdbcs_dev
