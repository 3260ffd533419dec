// Host controller of the MI355X hybrid LO-MSAC estimator.
//
// Semantics follow HybridLOMSAC::EstimateModel (src/hybrid_ransac.h:38-206) step for
// step; the difference is WHERE the work runs.  The reference draws one minimal
// sample, solves it and scores its models over all 3N residuals before drawing the
// next.  Here the controller replays the reference's two random streams
// (sampler mt19937, solver-selection/LO mt19937, both seeded with random_seed) to
// generate a *speculative batch* of B iterations, assuming no local optimisation
// happens inside the batch; the GPU solves every sample and scores every model of
// the batch in one pass; the host then scans the per-iteration best scores in
// order, reproducing the sequential decisions exactly.  The only event that
// invalidates the rest of a batch is an LO run (it consumes the selection stream);
// the controller then rewinds both streams to the end of that iteration, runs LO
// and starts the next batch there.  New-best events before lo_starting_iterations
// do not consume randomness and do not cut the batch.  Results are therefore
// independent of the batch size (tests/test_engine_gpu.py checks this).
//
// Local optimisation stays on the host (north star); its full-data sweeps
// (ScoreModel / GetInliers) run on the GPU through the single-model sweep kernel.
#include <fcntl.h>
#include <immintrin.h>
#include <signal.h>
#include <unistd.h>
#include "engine.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "../include/mp_score.h"
#include "../kernels/kernels.h"
#include "batch_draw.h"
#include "env.h"
#include "lo_sweep.h"
#include "rng.h"

namespace mp {

// kCompactLut[m]: the lane numbers of the set bits of the 4-bit mask m, ascending
// (inliers(): AVX2 stream compaction of the error rows)
alignas(16) static const int32_t kCompactLut[16][4] = {
    {0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0}, {2, 0, 0, 0}, {0, 2, 0, 0}, {1, 2, 0, 0}, {0, 1, 2, 0},
    {3, 0, 0, 0}, {0, 3, 0, 0}, {1, 3, 0, 0}, {0, 1, 3, 0}, {2, 3, 0, 0}, {0, 2, 3, 0}, {1, 2, 3, 0}, {0, 1, 2, 3}};

#define MP_HIP(expr)                                                                                                    \
    do {                                                                                                               \
        hipError_t e_ = (expr);                                                                                        \
        if (e_ != hipSuccess)                                                                                          \
            throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #expr);               \
    } while (0)

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

const double kMax = DBL_MAX;

// Minimal-sample batches and their drawing: batch_draw.h.  MADPOSE_SAMPLER_TWO_PASS=0
// keeps the draw-by-draw loop for hybrid batches too, MADPOSE_SAMPLER_SIMD=0 the scalar
// two passes (A/B; identical draws).
int sampler_mode() {
    static const int mode = [] {
        if (!env_flag("MADPOSE_SAMPLER_TWO_PASS", true)) return 0;
        return env_flag("MADPOSE_SAMPLER_SIMD", true) ? 2 : 1;
    }();
    return mode;
}

// Background sampler: draws the next speculative batch while the current one is on
// the GPU and the host replays it / runs LO.  The batch is kept only if the current
// one neither triggers LO nor terminates, so the worker can be told to give up.
class Sampler {
  public:
    Sampler() : th_([this] { loop(); }) {}
    ~Sampler() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
            abort_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // starts drawing B iterations from `from` into *g (the caller must not touch *g
    // or the slot memory until finish()/cancel() returned); `after` runs on the worker
    // once the batch is drawn (the post-LO speculation launches it on the GPU there)
    // chain (nullable): a second batch for the same job -- once *g is drawn (and `after`
    // ran), chain->B more iterations are drawn from where it ended into chain->g (the
    // post-LO speculation's successor, drawn while the LO runs)
    struct Chain {
        Batch *g;
        uint32_t B;
        int slot;
        int *smp;
        std::function<void()> after; // runs once it is drawn (launches it; nullable)
    };
    void start(const IterationStream &from, Batch *g, uint32_t B, int slot, int *smp,
               std::function<void()> after = nullptr, const Chain *chain = nullptr) {
        std::unique_lock<std::mutex> lk(mu_);
        if (busy_) { // a chained batch nobody asked for (chained()) is still being drawn
            abort_ = true;
            done_cv_.wait(lk, [this] { return !busy_; });
        }
        g2_ = chain ? chain->g : nullptr;
        B2_ = chain ? chain->B : 0;
        slot2_ = chain ? chain->slot : 0;
        smp2_ = chain ? chain->smp : nullptr;
        after2_ = chain ? chain->after : nullptr;
        ok2_ = false;
        after_ = std::move(after);
        err_ = nullptr;
        rs_ = from;
        g_ = g;
        B_ = B;
        slot_ = slot;
        smp_ = smp;
        abort_ = false;
        busy_ = busy1_ = true;
        ok_ = false;
        ++gen_;
        cv_.notify_all();
    }
    // after finish(): waits for the chained batch (the rest of the job); whether it was
    // drawn, *rs the stream state after it
    bool chained(IterationStream *rs) {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return !busy_; });
        if (err2_) std::rethrow_exception(err2_);
        if (ok2_) *rs = rs2_;
        return ok2_;
    }
    // waits for the batch (not for a chained one: that is drawn on while the caller reads
    // this one, until chained(), cancel() or the next start()); on success *rs is the
    // stream state after it
    bool finish(IterationStream *rs) {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return !busy1_; });
        if (err_) std::rethrow_exception(err_);
        if (ok_) *rs = rs1_;
        return ok_;
    }
    void cancel() {
        abort_ = true;
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return !busy_; });
    }

  private:
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
            if (quit_) return;
            seen = gen_;
            lk.unlock();
            const bool ok = draw_batch(rs_, *g_, B_, slot_, smp_, &abort_, sampler_mode());
            std::exception_ptr err;
            if (ok && after_) {
                try {
                    after_();
                } catch (...) {
                    err = std::current_exception();
                }
            }
            Batch *const g2 = g2_; // (set with the job, under the lock)
            lk.lock();
            rs1_ = rs_;
            err_ = err;
            ok_ = ok;
            busy1_ = false; // finish() returns here: the chained batch is drawn after it
            ok2_ = false;
            err2_ = nullptr;
            const bool go2 = ok && !err && g2;
            if (!go2) busy_ = false;
            done_cv_.notify_all();
            if (!go2) continue;
            lk.unlock();
            std::exception_ptr err2;
            IterationStream r2 = rs_;
            bool ok2 = draw_batch(r2, *g2, B2_, slot2_, smp2_, &abort_, sampler_mode());
            if (ok2 && after2_) {
                try {
                    after2_();
                } catch (...) {
                    err2 = std::current_exception();
                    ok2 = false;
                }
            }
            lk.lock();
            rs2_ = r2;
            ok2_ = ok2;
            err2_ = err2;
            busy_ = false;
            done_cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    IterationStream rs_;
    Batch *g_ = nullptr;
    uint32_t B_ = 0;
    int slot_ = 0;
    int *smp_ = nullptr;
    std::function<void()> after_;
    Batch *g2_ = nullptr;
    std::function<void()> after2_;
    uint32_t B2_ = 0;
    int slot2_ = 0;
    int *smp2_ = nullptr;
    IterationStream rs1_, rs2_; // the streams after the batch / after the chained one
    bool ok2_ = false;
    std::exception_ptr err_, err2_;
    std::atomic<bool> abort_{false};
    bool busy_ = false, busy1_ = false, ok_ = false, quit_ = false; // busy1_: the first batch is drawing
    uint64_t gen_ = 0;
    std::thread th_;
};

// ---------------------------------------------------------------------------
// Device resources of one LO lane (the estimator thread or an LO worker): a stream and
// the staging of the opt-in device LM (MADPOSE_DEVICE_LM).  The LO sweeps themselves
// run on the lane's own core (host/lo_sweep.h).
struct SweepSlot {
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // device-LM staging: job + index lists up, model + status down
    int64_t lm_cap = 0;
    char *h_lm = nullptr, *d_lm = nullptr;
    hipEvent_t lm_done = nullptr; // blocking-sync event: the waiting thread sleeps

    void ensure_lm(int64_t nidx) {
        if (!stream) {
            MP_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
            own_stream = true;
        }
        if (!lm_done) MP_HIP(hipEventCreateWithFlags(&lm_done, hipEventBlockingSync | hipEventDisableTiming));
        if (nidx <= lm_cap) return;
        if (h_lm) hipHostFree(h_lm);
        if (d_lm) hipFree(d_lm);
        h_lm = d_lm = nullptr;
        lm_cap = 0;
        const size_t bytes = lm_bytes(nidx);
        MP_HIP(hipHostMalloc(&h_lm, bytes, hipHostMallocDefault));
        MP_HIP(hipMalloc(&d_lm, bytes));
        lm_cap = nidx;
    }
    // layout: LmJob | Model out | int status | pad | int idx[nidx]
    static size_t lm_bytes(int64_t nidx) { return 512 + sizeof(int) * (size_t)nidx; }
};

int active_runs(int device);

// Worker threads for the parallel LO steps: run(n, f) calls f(job, lane) for jobs
// 0..n-1, lane 0 being the calling thread and lanes 1..size-1 the workers.  While the
// estimator has its device to itself, the workers spin (with pause, bounded by
// lo_spin_us() as the LM pool's) before they block, and so does the caller at the
// join: a futex wake-up per worker per LO delayed the steps of each LO by ~30 us
// (steps phase 230 us for a 200 us longest step, profiles/r04/lotab).  With other
// estimators on the device they block at once (their threads share the CPUs).
// MADPOSE_LO_WORKER_SPIN=0 turns the spinning off.
class LoWorkers {
  public:
    LoWorkers(int lanes, int device) : device_(device) {
        // microseconds (MADPOSE_LO_WORKER_SPIN; 0: block at once); default 2000 -- the
        // LO runs of a pair come ~0.3-1 ms apart, so a shorter spin sleeps through the
        // gap -- or 0 where the LM pool does not spin either (a small CPU share per rank)
        spin_ns_ = 1000ll * env_int("MADPOSE_LO_WORKER_SPIN", lo_spin_us() > 0 ? 2000 : 0, 0, 1000000);
        for (int i = 1; i < lanes; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~LoWorkers() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_.store(true);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int lanes() const { return (int)th_.size() + 1; }
    void run(int n, const std::function<void(int, int)> &f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            f_ = &f;
            n_ = n;
            next_.store(0);
            active_.store((int)th_.size());
            err_ = nullptr;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work(0);
        if (!spin_until([this] { return active_.load(std::memory_order_acquire) == 0; })) {
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [this] { return active_.load(std::memory_order_acquire) == 0; });
        }
        f_ = nullptr;
        if (err_) std::rethrow_exception(err_);
    }

  private:
    // polls ready() with pause for at most spin_ns_ (none with other estimators on the
    // device); true once it held
    template <class F> bool spin_until(const F &ready) const {
        if (spin_ns_ <= 0 || active_runs(device_) > 1) return ready();
        const auto t0 = Clock::now();
        for (int k = 0;; ++k) {
            if (ready()) return true;
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
            if ((k & 63) == 63 &&
                std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count() > spin_ns_)
                return ready();
        }
    }
    void work(int lane) {
        for (int k; (k = next_.fetch_add(1)) < n_;) {
            try {
                (*f_)(k, lane);
            } catch (...) {
                std::lock_guard<std::mutex> lk(err_mu_);
                if (!err_) err_ = std::current_exception();
            }
        }
    }
    void loop(int lane) {
        uint64_t seen = 0;
        for (;;) {
            if (!spin_until([&] { return quit_.load() || gen_.load(std::memory_order_acquire) != seen; })) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_.load() || gen_.load(std::memory_order_acquire) != seen; });
            }
            {
                std::lock_guard<std::mutex> lk(mu_); // (pairs with run()'s publication)
                if (quit_.load()) return;
                seen = gen_.load(std::memory_order_relaxed);
            }
            work(lane);
            if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, err_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int, int)> *f_ = nullptr;
    int n_ = 0;
    std::atomic<int> active_{0};
    std::atomic<int> next_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> quit_{false};
    std::exception_ptr err_;
    int device_ = 0;
    long long spin_ns_ = 0;
};

constexpr int kLoLanes = 12; // most concurrent LO steps (and sweep slots) per context

// concurrent LO steps of one estimator (MADPOSE_LO_LANES, 1..kLoLanes): the default
// is 4 lanes; see DESIGN.md §8 for the measurements behind it
inline int lo_lanes_setting() {
    static const int v = [] {
        return (int)env_int("MADPOSE_LO_LANES", 4, 1, kLoLanes);
    }();
    return v;
}

// ---------------------------------------------------------------------------
// Device context: stream + cached buffers (one per device and concurrent caller)
//
// The per-batch buffers come in two slots (BatchBufs), the slot of a batch being the
// host sample slot it was drawn into: the continuation batch is launched into the other
// slot while the host still reads this one's results (early continuation, Run::run).
struct BatchBufs {
    int *d_counts = nullptr;
    IterResult *d_res = nullptr;
    int *d_work = nullptr, *h_work = nullptr; // score_batch's evaluated (model, trip) pairs per iteration
    // the walk's inputs (ScoreBound::flags8 / cand_out): one byte per iteration (model
    // count | 0x80 for a possible new best), copied back; the IterResults of the marked
    // iterations, written by score_batch into mapped memory
    uint8_t *d_flags8 = nullptr, *h_flags8 = nullptr;
    IterResult *h_cand = nullptr, *d_cand = nullptr;

    Model *d_models = nullptr;
    ScoreRec *d_recs = nullptr;
    double *d_scores = nullptr;
    // score_batch writes the models of the iterations that beat the pre-batch best here
    // (mapped pinned memory, one slot per iteration of the batch)
    Model *h_recmodel = nullptr, *d_recmodel = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr}; // solve start / score start / score end
    hipEvent_t ev_fork = nullptr, ev_join = nullptr; // MD side stream fork / join
    hipEvent_t ev_h2d = nullptr;                    // the batch's samples have been copied
    hipEvent_t ev_solved = nullptr;                 // the batch's solver kernels are done
    hipEvent_t ev_done = nullptr;                   // the batch's results are on the host
    // each slot's batches run on the slot's stream from the slot's sample buffer: a
    // continuation in the other slot solves while this slot's batch is scored (it waits
    // for this slot's ev_solved first: the point solvers' workspace and the MD side
    // stream are shared)
    hipStream_t stream = nullptr;
    int *d_samples = nullptr;
    unsigned epoch_hi = 0;                          // ~epoch of the batch last launched here
    bool h2d_pending = false;                       // launched, ev_h2d not yet waited for
};

struct DeviceCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t cap_n = 0;
    int cap_b = 0, cap_m = 0;
    double *d_pair = nullptr; // 12 arrays of cap_n (PairData)
    // score_batch's record word (kernels.hip ScoreBound::rec) and the batch epoch
    unsigned long long *d_recword = nullptr;
    uint32_t epoch = 0;
    BatchBufs bb[2];
    ScoreRec *d_rec1 = nullptr;
    double *d_err = nullptr, *d_score1 = nullptr;
    // staged point-solver workspace (kernels.h PtWorkspace)
    double *d_pt_cand = nullptr, *d_pt_pen = nullptr;
    int *d_pt_ncand = nullptr, *d_pt_valid = nullptr;
    Model *d_pt_slots = nullptr;
    // the two-stage exact MD solver's per-sample state (kernels.h kMdWsStride, SoA, ld cap_b)
    double *d_md_ws = nullptr;
    int *d_md_nr = nullptr;
    // device resources of the LO lanes (lane 0: the estimator thread)
    SweepSlot sweep_slot[kLoLanes];
    std::unique_ptr<LoWorkers> lo_workers; // created on first parallel LO
    // pinned host mirrors
    int *h_samples = nullptr; // two slots of 9 * max_batch ints
    double *h_err = nullptr, *h_score1 = nullptr;
    ScoreRec *h_rec1 = nullptr;
    Model *h_model1 = nullptr;
    // the MD solver runs on md_stream, concurrently with the point-solver stages; host
    // reads of a finished batch's device data go through copy_stream (the main stream
    // may already hold the next batch)
    hipStream_t md_stream = nullptr, copy_stream = nullptr;
    std::unique_ptr<Sampler> sampler;               // created on first use

    void free_all() {
        hipSetDevice(device);
        for (void *p : {(void *)d_pair, (void *)bb[0].d_samples, (void *)bb[1].d_samples, (void *)d_recword, (void *)d_rec1, (void *)d_err,
                        (void *)d_score1, (void *)d_pt_cand, (void *)d_pt_pen, (void *)d_pt_ncand, (void *)d_pt_valid,
                        (void *)d_pt_slots, (void *)d_md_ws, (void *)d_md_nr})
            if (p) hipFree(p);
        for (void *p : {(void *)h_samples, (void *)h_err, (void *)h_score1, (void *)h_rec1, (void *)h_model1})
            if (p) hipHostFree(p);
        for (BatchBufs &q : bb) {
            for (void *p : {(void *)q.d_counts, (void *)q.d_res, (void *)q.d_work, (void *)q.d_models,
                            (void *)q.d_recs, (void *)q.d_scores, (void *)q.d_flags8})
                if (p) hipFree(p);
            for (void *p : {(void *)q.h_flags8, (void *)q.h_cand, (void *)q.h_work, (void *)q.h_recmodel})
                if (p) hipHostFree(p);
            q.d_counts = q.d_work = q.h_work = nullptr;
            q.d_res = q.h_cand = q.d_cand = nullptr;
            q.d_flags8 = q.h_flags8 = nullptr;
            q.d_models = q.h_recmodel = q.d_recmodel = nullptr;
            q.d_recs = nullptr;
            q.d_scores = nullptr;
            q.h2d_pending = false;
        }
        d_pair = d_err = d_score1 = nullptr;
        bb[0].d_samples = bb[1].d_samples = nullptr;
        d_recword = nullptr;
        d_rec1 = nullptr;
        d_pt_cand = d_pt_pen = nullptr;
        d_pt_ncand = d_pt_valid = nullptr;
        d_pt_slots = nullptr;
        d_md_ws = nullptr;
        d_md_nr = nullptr;
        h_samples = nullptr;
        h_err = h_score1 = nullptr;
        h_rec1 = nullptr;
        h_model1 = nullptr;
        cap_n = 0;
        cap_b = cap_m = 0;
    }

    void ensure(int64_t n, int B, int M) {
        if (n <= cap_n && B <= cap_b && M <= cap_m) return;
        const int64_t nn = std::max<int64_t>(std::max<int64_t>(n, cap_n), 64);
        const int bb_ = std::max(B, cap_b), mm = std::max(M, cap_m);
        MP_HIP(hipSetDevice(device));
        MP_HIP(hipDeviceSynchronize()); // (an early continuation may still use the old buffers)
        free_all();
        MP_HIP(hipMalloc(&d_pair, sizeof(double) * 12 * nn));
        MP_HIP(hipMalloc(&d_err, sizeof(double) * 3 * nn));
        for (BatchBufs &q : bb) MP_HIP(hipMalloc(&q.d_samples, sizeof(int) * 9 * bb_));
        MP_HIP(hipMalloc(&d_recword, sizeof(unsigned long long)));
        MP_HIP(hipMemset(d_recword, 0xff, sizeof(unsigned long long)));
        for (BatchBufs &q : bb) {
            MP_HIP(hipMalloc(&q.d_counts, sizeof(int) * bb_));
            MP_HIP(hipMalloc(&q.d_res, sizeof(IterResult) * bb_));
            MP_HIP(hipMalloc(&q.d_work, sizeof(int) * bb_));
            MP_HIP(hipMalloc(&q.d_models, sizeof(Model) * (size_t)bb_ * mm));
            MP_HIP(hipMalloc(&q.d_recs, sizeof(ScoreRec) * (size_t)bb_ * mm));
            MP_HIP(hipMalloc(&q.d_scores, sizeof(double) * (size_t)bb_ * mm));
            // (score_batch writes a byte per iteration to device memory and one copy
            // brings them over; writing every workgroup's result to mapped host memory
            // made the kernel 51 -> 63 us per cal launch, profiles/r05/r5j -- only the
            // few marked iterations write theirs there)
            MP_HIP(hipMalloc(&q.d_flags8, (size_t)bb_));
            MP_HIP(hipHostMalloc(&q.h_flags8, (size_t)bb_, hipHostMallocDefault));
            MP_HIP(hipHostMalloc(&q.h_cand, sizeof(IterResult) * bb_, hipHostMallocMapped | hipHostMallocCoherent));
            MP_HIP(hipHostGetDevicePointer((void **)&q.d_cand, q.h_cand, 0));
            MP_HIP(hipHostMalloc(&q.h_work, sizeof(int) * bb_, hipHostMallocDefault));
            MP_HIP(hipHostMalloc(&q.h_recmodel, sizeof(Model) * (size_t)bb_,
                                 hipHostMallocMapped | hipHostMallocCoherent));
            MP_HIP(hipHostGetDevicePointer((void **)&q.d_recmodel, q.h_recmodel, 0));
        }
        MP_HIP(hipMalloc(&d_rec1, sizeof(ScoreRec) * 64));
        MP_HIP(hipMalloc(&d_pt_cand, sizeof(double) * (size_t)bb_ * kPtCandStride));
        // (the pencil workspace of the shared-focal root stage; a stub elsewhere)
        MP_HIP(hipMalloc(&d_pt_pen, sizeof(double) * (mm == kMaxModelsSF ? (size_t)bb_ * kPtPenStride : 1)));
        MP_HIP(hipMalloc(&d_pt_ncand, sizeof(int) * (size_t)bb_));
        MP_HIP(hipMalloc(&d_pt_valid, sizeof(int) * (size_t)bb_ * kPtSlotStride));
        MP_HIP(hipMalloc(&d_pt_slots, sizeof(Model) * (size_t)bb_ * kPtSlotStride));
        MP_HIP(hipMalloc(&d_md_ws, sizeof(double) * (size_t)bb_ * kMdWsStride));
        MP_HIP(hipMalloc(&d_md_nr, sizeof(int) * (size_t)bb_));
        MP_HIP(hipMalloc(&d_score1, sizeof(double) * 64));
        // two slots each: the next batch is generated while the current one is in flight
        MP_HIP(hipHostMalloc(&h_samples, sizeof(int) * 2 * 9 * bb_, hipHostMallocDefault));
        MP_HIP(hipHostMalloc(&h_err, sizeof(double) * 3 * nn, hipHostMallocDefault));
        MP_HIP(hipHostMalloc(&h_score1, sizeof(double) * 64, hipHostMallocDefault));
        MP_HIP(hipHostMalloc(&h_rec1, sizeof(ScoreRec) * 64, hipHostMallocDefault));
        MP_HIP(hipHostMalloc(&h_model1, sizeof(Model) * 64, hipHostMallocDefault));
        cap_n = nn;
        cap_b = bb_;
        cap_m = mm;
    }
};

std::mutex g_pool_mu;
std::vector<DeviceCtx *> g_pool;

// Process teardown: the pooled (idle) contexts' host threads -- each context's sampler
// and LO workers -- are stopped and joined before the HIP runtime's own teardown (this
// library's static destructors run first: it is loaded after libamdhip64).  A context
// leased by an estimator still running at exit is not in the pool and is left alone.
// The device buffers are not freed: the process is ending.
struct PoolReaper {
    ~PoolReaper() {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (DeviceCtx *c : g_pool) {
            c->sampler.reset();
            c->lo_workers.reset();
        }
    }
} g_pool_reaper;

// MADPOSE_SEGV_MAPS (diagnostic, presence): on SIGSEGV / SIGBUS write the fault address
// and /proc/self/maps to stderr, then hand the signal to the handler installed before
// (a profiler's stack printer, or the default action).  Async-signal-safe: open / read /
// write only.
struct sigaction g_old_segv, g_old_bus;
void segv_maps_handler(int sig, siginfo_t *si, void *uc) {
    char buf[4096];
    static const char hex[] = "0123456789abcdef";
    int k = 0;
    const char *hdr = "[madpose] fault address 0x";
    while (*hdr) buf[k++] = *hdr++;
    const unsigned long long a = (unsigned long long)(uintptr_t)(si ? si->si_addr : nullptr);
    for (int sh = 60; sh >= 0; sh -= 4) buf[k++] = hex[(a >> sh) & 15];
    const char *tail = ", /proc/self/maps:\n";
    while (*tail) buf[k++] = *tail++;
    ssize_t w = write(2, buf, (size_t)k);
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        ssize_t r;
        while ((r = read(fd, buf, sizeof(buf))) > 0) w = write(2, buf, (size_t)r);
        close(fd);
    }
    (void)w;
    const struct sigaction &old = sig == SIGBUS ? g_old_bus : g_old_segv;
    if (old.sa_flags & SA_SIGINFO) {
        old.sa_sigaction(sig, si, uc);
    } else if (old.sa_handler != SIG_IGN && old.sa_handler != SIG_DFL) {
        old.sa_handler(sig);
    } else {
        signal(sig, SIG_DFL);
        raise(sig);
    }
}
void install_segv_maps() {
    static std::once_flag once;
    std::call_once(once, [] {
        if (!std::getenv("MADPOSE_SEGV_MAPS")) return;
        struct sigaction sa;
        std::memset(&sa, 0, sizeof(sa));
        sa.sa_sigaction = segv_maps_handler;
        sa.sa_flags = SA_SIGINFO;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGSEGV, &sa, &g_old_segv);
        sigaction(SIGBUS, &sa, &g_old_bus);
    });
}

std::atomic<bool> g_prof_on{false};
std::mutex g_prof_mu;
KernelProfile g_prof;

// estimators running on each device (leases held): the early continuation is
// speculative GPU work that pays only while one estimator has the device to itself
constexpr int kMaxDevices = 64;
std::atomic<int> g_active_runs[kMaxDevices];
int active_runs(int device) {
    return device >= 0 && device < kMaxDevices ? g_active_runs[device].load(std::memory_order_relaxed) : 1;
}

struct CtxLease {
    DeviceCtx *c = nullptr;
    explicit CtxLease(int device) {
        install_segv_maps();
        {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            for (size_t i = 0; i < g_pool.size(); ++i)
                if (g_pool[i]->device == device) {
                    c = g_pool[i];
                    g_pool.erase(g_pool.begin() + i);
                    break;
                }
        }
        if (!c) {
            int cnt = 0;
            if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
                throw std::runtime_error("no HIP device available (MI355X required; there is no CPU fallback)");
            if (device < 0 || device >= cnt) throw std::invalid_argument("device index out of range");
            c = new DeviceCtx();
            c->device = device;
            MP_HIP(hipSetDevice(device));
            MP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            MP_HIP(hipStreamCreateWithFlags(&c->md_stream, hipStreamNonBlocking));
            MP_HIP(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
            c->bb[0].stream = c->stream;
            MP_HIP(hipStreamCreateWithFlags(&c->bb[1].stream, hipStreamNonBlocking));
            for (BatchBufs &q : c->bb) {
                for (auto &e : q.ev) MP_HIP(hipEventCreate(&e));
                MP_HIP(hipEventCreateWithFlags(&q.ev_solved, hipEventDisableTiming));
                MP_HIP(hipEventCreateWithFlags(&q.ev_fork, hipEventDisableTiming));
                MP_HIP(hipEventCreateWithFlags(&q.ev_join, hipEventDisableTiming));
                MP_HIP(hipEventCreateWithFlags(&q.ev_h2d, hipEventDisableTiming));
                MP_HIP(hipEventCreateWithFlags(&q.ev_done, hipEventDisableTiming));
            }
        }
        MP_HIP(hipSetDevice(device));
        if (device < kMaxDevices) g_active_runs[device].fetch_add(1, std::memory_order_relaxed);
    }
    ~CtxLease() {
        if (c->device < kMaxDevices) g_active_runs[c->device].fetch_sub(1, std::memory_order_relaxed);
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool.push_back(c);
    }
};

// ---------------------------------------------------------------------------
void inv3(const double *K, double *Ki) {
    // no FMA contraction: the calibrated rays K^-1 x the MD solvers see are the oracle's
    // (oracle/src/estimator.cpp inv3, mv3) to the bit
#pragma clang fp contract(off)
    const double d = K[0] * (K[4] * K[8] - K[5] * K[7]) - K[1] * (K[3] * K[8] - K[5] * K[6]) +
                     K[2] * (K[3] * K[7] - K[4] * K[6]);
    Ki[0] = (K[4] * K[8] - K[5] * K[7]) / d;
    Ki[1] = (K[2] * K[7] - K[1] * K[8]) / d;
    Ki[2] = (K[1] * K[5] - K[2] * K[4]) / d;
    Ki[3] = (K[5] * K[6] - K[3] * K[8]) / d;
    Ki[4] = (K[0] * K[8] - K[2] * K[6]) / d;
    Ki[5] = (K[2] * K[3] - K[0] * K[5]) / d;
    Ki[6] = (K[3] * K[7] - K[4] * K[6]) / d;
    Ki[7] = (K[1] * K[6] - K[0] * K[7]) / d;
    Ki[8] = (K[0] * K[4] - K[1] * K[3]) / d;
}

// Problem setup shared by every entry point: the option transform to three data
// types (src/hybrid_pose_estimator.cpp:13-23) and, for SF/TF, pp-centring plus
// PoseLib normalize_points(..., true, false, true) (..shared..cpp:14-25).
struct Problem {
    PairConst C;
    HostPair H;
    double norm_scale = 1.0;
};

// Ceres settings of one LeastSquares / NonMinimalSolver call (the flags of
// Run::least_squares; src/hybrid_pose_estimator.cpp:203, 281 and the SF/TF analogues)
LmJob make_lm_job(const Problem &P, const EstimatorConfig &cfg, const int *sizes, int off, bool nonminimal,
                  const Model &m) {
    LmJob J;
    std::memset(&J, 0, sizeof(J));
    const bool use_reproj = cfg.lo_type != 1, use_sampson = cfg.lo_type != 2;
    const int v = P.C.variant;
    J.off0 = off;
    J.n0 = use_reproj ? sizes[0] : 0;
    J.off1 = off + sizes[0];
    J.n1 = use_reproj ? sizes[1] : 0;
    J.off2 = off + sizes[0] + sizes[1];
    J.n2 = use_sampson ? sizes[2] : 0;
    J.use_shift = (v == kCal || (v == kSF && nonminimal)) ? cfg.use_shift : 1;
    J.min_depth_constraint = cfg.min_depth_constraint;
    if (P.C.scale_only) { // HybridPoseOptimizerScaleOnly: offsets constant, unbounded
        J.use_shift = 0;
        J.min_depth_constraint = 0;
    }
    J.w_sampson = v == kCal ? std::sqrt(P.H.sampson_squared_weight) /
                                  (1.0 / (P.C.K0[0] + P.C.K0[4]) + 1.0 / (P.C.K1[0] + P.C.K1[4]))
                            : std::sqrt(P.H.sampson_squared_weight);
    J.ftol = cfg.ftol;
    J.gtol = cfg.gtol;
    J.ptol = cfg.ptol;
    J.max_iter = (int)cfg.max_iter;
    J.nonmonotonic = cfg.nonmonotonic ? 1 : 0;
    J.m = m;
    return J;
}

// The pair's magnitudes behind the screening margins (PairConst::ea.., mp_score.h
// score_margins): maxima of the rays' absolute sums, depths and coordinates.
void pair_magnitudes(PairConst &C, const HostPair &H) {
    const bool cal = C.variant == kCal;
    double ea = 0, eap = 0, exi = 0, eb = 0, ebp = 0, exj = 0, ed0 = 0, ed1 = 0, ex0 = 0, ex1 = 0, eab2 = 0;
    for (int i = 0; i < H.n; ++i) {
        const double u0 = H.x0[2 * i], v0 = H.x0[2 * i + 1], u1 = H.x1[2 * i], v1 = H.x1[2 * i + 1];
        ex0 = std::max(ex0, std::max(std::fabs(u0), std::fabs(v0)));
        ex1 = std::max(ex1, std::max(std::fabs(u1), std::fabs(v1)));
        ed0 = std::max(ed0, std::fabs(H.d0[i]));
        ed1 = std::max(ed1, std::fabs(H.d1[i]));
        if (cal) {
            auto ray = [](const double *Ki, double u, double v, double *abs1, double *absp, double *xi) {
                double a[3], p = 0.0;
                for (int j = 0; j < 3; ++j) {
                    a[j] = Ki[3 * j] * u + Ki[3 * j + 1] * v + Ki[3 * j + 2];
                    p += std::fabs(Ki[3 * j] * u) + std::fabs(Ki[3 * j + 1] * v) + std::fabs(Ki[3 * j + 2]);
                }
                *abs1 = std::max(*abs1, std::fabs(a[0]) + std::fabs(a[1]) + std::fabs(a[2]));
                *absp = std::max(*absp, p);
                *xi = std::max(*xi, p / (std::fabs(a[0]) + std::fabs(a[1]) + 1.0));
            };
            ray(C.K0i, u0, v0, &ea, &eap, &exi);
            ray(C.K1i, u1, v1, &eb, &ebp, &exj);
            const double a0 = C.K0i[0] * u0 + C.K0i[1] * v0 + C.K0i[2], a1 = C.K0i[3] * u0 + C.K0i[4] * v0 + C.K0i[5];
            const double b0 = C.K1i[0] * u1 + C.K1i[1] * v1 + C.K1i[2], b1 = C.K1i[3] * u1 + C.K1i[4] * v1 + C.K1i[5];
            const double ab = (std::fabs(a0) + std::fabs(a1) + 1.0) * (std::fabs(b0) + std::fabs(b1) + 1.0);
            eab2 = std::max(eab2, ab * ab);
        } else {
            ea = std::max(ea, std::fabs(u0) + std::fabs(v0));
            eb = std::max(eb, std::fabs(u1) + std::fabs(v1));
            const double ab = (std::fabs(u0) + std::fabs(v0) + 1.0) * (std::fabs(u1) + std::fabs(v1) + 1.0);
            eab2 = std::max(eab2, ab * ab);
        }
    }
    if (!cal) {
        eap = ea;
        ebp = eb;
    }
    // (a non-finite coordinate or depth turns screening off: make_problem)
    C.ea = ea * (1 + 1e-12);
    C.eap = eap * (1 + 1e-12);
    C.exi = exi * (1 + 1e-12);
    C.eb = eb * (1 + 1e-12);
    C.ebp = ebp * (1 + 1e-12);
    C.exj = exj * (1 + 1e-12);
    C.ed0 = ed0;
    C.ed1 = ed1;
    C.ex0 = ex0;
    C.ex1 = ex1;
    C.eab2 = eab2 * (1 + 1e-12);
}

Problem make_problem(const PairInput &in, const RansacOptions &o, const EstimatorConfig &cfg) {
    // no FMA contraction: the normalization scale (and with it every normalized
    // coordinate the MD solvers see) is the oracle's to the bit (estimator.cpp:88-103)
#pragma clang fp contract(off)
    Problem P;
    const int n = (int)in.n;
    PairConst &C = P.C;
    std::memset(&C, 0, sizeof(C));
    // the scale-only estimator runs on the calibrated geometry (src/hybrid_pose_estimator.h:110-134)
    C.scale_only = in.variant == kScaleOnly ? 1 : 0;
    C.variant = C.scale_only ? kCal : in.variant;
    C.n = n;
    C.score_type = cfg.score_type;
    C.min_depth_constraint = cfg.min_depth_constraint ? 1 : 0;
    C.use_shift = cfg.use_shift ? 1 : 0;
    // option-gated MD alternates (src/hybrid_pose_estimator.cpp:75-78, ..shared..cpp:62-65,
    // ..two..cpp:87-94); use_ours wins over use_4p4d, 4p4d exists for two-focal only
    C.md_alt = C.scale_only ? 0 : (o.use_ours ? 1 : ((o.use_4p4d && in.variant == kTF) ? 2 : 0));
    C.min_depth[0] = in.min_depth[0];
    C.min_depth[1] = in.min_depth[1];
    HostPair &H = P.H;
    H.variant = C.variant;
    H.n = n;
    H.x0.resize(2 * n);
    H.x1.resize(2 * n);
    H.d0.assign(in.d0, in.d0 + n);
    H.d1.assign(in.d1, in.d1 + n);
    H.min_depth[0] = in.min_depth[0];
    H.min_depth[1] = in.min_depth[1];
    double thr0 = o.squared_inlier_thresholds[0], thr1 = o.squared_inlier_thresholds[1];
    if (C.variant == kCal) {
        std::memcpy(C.K0, in.cam0, sizeof(C.K0));
        std::memcpy(C.K1, in.cam1, sizeof(C.K1));
        inv3(C.K0, C.K0i);
        inv3(C.K1, C.K1i);
        std::memcpy(H.x0.data(), in.x0, sizeof(double) * 2 * n);
        std::memcpy(H.x1.data(), in.x1, sizeof(double) * 2 * n);
        const double s = 1.0 / (C.K0[0] + C.K0[4]) + 1.0 / (C.K1[0] + C.K1[4]);
        C.loss_scale = 1.0 / (s * s);
        // upper-triangular intrinsics with unit last row: the score kernels' ray form
        auto tri = [](const double *K) { return K[3] == 0.0 && K[6] == 0.0 && K[7] == 0.0 && K[8] == 1.0; };
        C.kstd = (tri(C.K0) && tri(C.K1) && tri(C.K0i) && tri(C.K1i)) ? 1 : 0;
    } else {
        double scale = 0.0;
        for (int i = 0; i < n; ++i) {
            const double a0 = in.x0[2 * i] - in.cam0[0], a1 = in.x0[2 * i + 1] - in.cam0[1];
            const double b0 = in.x1[2 * i] - in.cam1[0], b1 = in.x1[2 * i + 1] - in.cam1[1];
            H.x0[2 * i] = a0;
            H.x0[2 * i + 1] = a1;
            H.x1[2 * i] = b0;
            H.x1[2 * i + 1] = b1;
            // (two accumulations per correspondence, as PoseLib's normalize_points and the
            // oracle: the scale, hence every normalized coordinate, to the bit)
            scale += std::sqrt(a0 * a0 + a1 * a1);
            scale += std::sqrt(b0 * b0 + b1 * b1);
        }
        scale = (n > 0) ? scale / (std::sqrt(2.0) * n) : 1.0;
        for (int i = 0; i < 2 * n; ++i) {
            H.x0[i] /= scale;
            H.x1[i] /= scale;
        }
        P.norm_scale = scale;
        thr0 /= scale * scale;
        thr1 /= scale * scale;
        for (int i = 0; i < 9; ++i) C.K0[i] = C.K1[i] = C.K0i[i] = C.K1i[i] = (i % 4 == 0) ? 1.0 : 0.0;
        C.loss_scale = 1.0;
    }
    pair_magnitudes(C, H);
    {
        C.tie_scale = env_real("MADPOSE_TIE_SCALE", 1.0, 1.0, 1e300);
        // a non-finite coordinate or depth: no screening at all (every margin infinite;
        // the score kernel's residuals could be NaN where no gate flags them)
        bool finite = true;
        for (int i = 0; i < 2 * n && finite; ++i) finite = std::isfinite(H.x0[i]) && std::isfinite(H.x1[i]);
        for (int i = 0; i < n && finite; ++i) finite = std::isfinite(H.d0[i]) && std::isfinite(H.d1[i]);
        if (!finite) C.tie_scale = std::numeric_limits<double>::infinity();
    }
    std::memcpy(H.K0, C.K0, sizeof(H.K0));
    std::memcpy(H.K1, C.K1, sizeof(H.K1));
    std::memcpy(H.K0i, C.K0i, sizeof(H.K0i));
    std::memcpy(H.K1i, C.K1i, sizeof(H.K1i));
    const double w0 = o.data_type_weights[0];
    // data_type_weights_[1] *= 2 * thr0 / thr1 (src/hybrid_pose_estimator.cpp:16-17)
    const double ws = o.data_type_weights[1] * (2 * thr0 / thr1);
    H.sampson_squared_weight = ws;
    C.thr[0] = C.thr[1] = thr0;
    C.thr[2] = thr1;
    C.w[0] = C.w[1] = w0;
    C.w[2] = ws;
    margin_consts(C);
    return P;
}

void upload_pair(DeviceCtx &X, const Problem &P, PairData *D) {
    const int64_t n = P.C.n;
    double *base = X.d_pair;
    const int64_t cn = X.cap_n;
    // one upload: the six arrays packed at stride n on the host, placed at their device
    // stride cap_n by one 2-D copy (the pooled context's cap_n is the high-water mark of
    // the pairs it has seen: a small pair after a large one moves 6 n doubles, not 6 cap_n)
    if (n > cn) throw std::logic_error("upload_pair: pair larger than the device buffers");
    std::vector<double> soa(6 * (size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        soa[i] = P.H.x0[2 * i];
        soa[n + i] = P.H.x0[2 * i + 1];
        soa[2 * n + i] = P.H.x1[2 * i];
        soa[3 * n + i] = P.H.x1[2 * i + 1];
        soa[4 * n + i] = P.H.d0[i];
        soa[5 * n + i] = P.H.d1[i];
    }
    if (n > 0)
        MP_HIP(hipMemcpy2DAsync(base, sizeof(double) * (size_t)cn, soa.data(), sizeof(double) * (size_t)n,
                                sizeof(double) * (size_t)n, 6, hipMemcpyHostToDevice, X.stream));
    D->x0u = base;
    D->x0v = base + cn;
    D->x1u = base + 2 * cn;
    D->x1v = base + 3 * cn;
    D->d0 = base + 4 * cn;
    D->d1 = base + 5 * cn;
    D->r0 = base + 6 * cn;
    D->r1 = base + 7 * cn;
    D->a0 = base + 8 * cn;
    D->a1 = base + 9 * cn;
    D->b0 = base + 10 * cn;
    D->b1 = base + 11 * cn;
    MP_HIP(launch_prep_pair(X.stream, P.C, *D, base + 6 * cn, base + 7 * cn, base + 8 * cn, base + 9 * cn,
                            base + 10 * cn, base + 11 * cn));
    // the staging vector dies here: make the copies complete first
    MP_HIP(hipStreamSynchronize(X.stream));
}

// ---------------------------------------------------------------------------
// The estimator run (one pair)
class Run {
  public:
    Run(DeviceCtx &X, const Problem &P, const RansacOptions &o, const EstimatorConfig &cfg)
        : X_(X), P_(P), o_(o), cfg_(cfg), n_(P.C.n), variant_(P.C.variant), maxm_(max_models(P.C.variant)) {
        const int kmd = variant_ == kCal ? 3 : 4;
        const int kpt = variant_ == kCal ? 5 : (variant_ == kSF ? 6 : 7);
        ss_[0][0] = kmd;
        ss_[0][1] = kmd;
        ss_[0][2] = 0;
        ss_[1][0] = 0;
        ss_[1][1] = 0;
        ss_[1][2] = kpt;
        min_sample_size_ = kpt;
        non_min_sample_size_ = variant_ == kCal ? 35 : 36;
        thr_[0] = P.C.thr[0];
        thr_[1] = P.C.thr[1];
        thr_[2] = P.C.thr[2];
        w_[0] = P.C.w[0];
        w_[1] = P.C.w[1];
        w_[2] = P.C.w[2];
        max_batch_ = (int)env_int("MADPOSE_MAX_BATCH", 32768, 1, 1 << 22);
        // (1024: the solver kernels cost about the same at 128 and at 1024 samples, so a
        // short run -- the ScanNet stand-in's 1000 iterations -- takes fewer round trips:
        // 903 / 982 / 998 pairs/s at 128 / 512 / 1000 on one box, profiles/r03/s6)
        // calibrated: 4096 since the post-LO speculation runs beside the LO (§2 step 6): a
        // bigger speculative batch costs no wait and covers more iterations per LO cycle,
        // 4.31 -> 4.07 ms per pair (2048: 4.19; profiles/r05/min_batch); shared focal
        // neutral at 2048 (9.94 -> 9.97 ms)
        min_batch_ = (int)env_int("MADPOSE_MIN_BATCH", variant_ == kCal ? 4096 : 1024, 1, 1 << 22);
        min_batch_ = std::min(min_batch_, max_batch_);
        // growth 1 for every variant: round 4 ran the shared focal at 2 (fewer, larger
        // batches for its latency-bound chain: 11.48 -> 10.97-11.20 ms, profiles/r04/gab2)
        // at 1.49 solved per accepted hypothesis; with the round-5 host the difference is
        // 10.62 (1.33) against 10.39 ms (1.42), 1.5: 10.50 (1.38), 3 x 60 pairs on one
        // box (profiles/r05/r5sg).  For cal, 0.5 and the waste it saves cost more round
        // trips than they save work (r04 gab)
        growth_ = env_real("MADPOSE_BATCH_GROWTH", 1.0, 0.01, 1e6);
        trace_ = std::getenv("MADPOSE_TRACE") != nullptr;
    }

    void run(Model *best, Stats *S);

  private:
    DeviceCtx &X_;
    const Problem &P_;
    const RansacOptions &o_;
    const EstimatorConfig &cfg_;
    const int n_, variant_, maxm_;
    int ss_[2][3];
    int min_sample_size_, non_min_sample_size_;
    double thr_[3], w_[3];
    int max_batch_, min_batch_;
    double growth_; // batch = growth_ x iterations so far (MADPOSE_BATCH_GROWTH)
    bool trace_ = false;
    // New bests are decided on reference-order sums (exact_score); score_batch's sums
    // screen with per-model margins (ScoreRec::tie, mp_score.h score_margins: |device
    // sum - reference-order sum| <= tie unless the iteration is flagged uncertain), see
    // the walk in run().  MADPOSE_TIE_SCALE multiplies every margin (tests force the
    // resolution path with a large factor).
    uint64_t tie_checks_ = 0;
    // MADPOSE_COUNT_DUMP=<file>: one line per walked iteration (iteration, solver type,
    // model count, the solver's sample) -- a diagnostic (tools/diag_counts.py)
    FILE *count_dump_ = nullptr;
    // MADPOSE_MODEL_DUMP=<file>: per walked iteration (int32 iteration, int32 model count,
    // the models as 17 doubles each, problem units) -- the oracle replays them
    // (ORACLE_MODEL_REPLAY, oracle/src/ransac.cpp) to separate the selection logic from
    // the solvers' rounding (tests/test_ties_gpu.py)
    FILE *model_dump_ = nullptr;
    // MADPOSE_TIMELINE=k (or k-m): the k-th estimator run of the process (0-based) prints its
    // timeline to stderr at the end -- one line per event, microseconds since the run
    // started: launch begin/end (B), wait begin/end, LO begin / prefix end / end, resolve
    // and exact-score calls, sampler joins -- a diagnostic of the critical path
    struct Timeline {
        bool on = false;
        long run = 0;
        Clock::time_point t0;
        struct Ev {
            double us;
            const char *what;
            long a;
        };
        std::vector<Ev> ev;
        std::mutex mu; // (the sampler thread launches speculative batches)
        void mark(const char *what, long a = 0) {
            if (!on) return;
            std::lock_guard<std::mutex> lk(mu);
            ev.push_back({1e6 * std::chrono::duration<double>(Clock::now() - t0).count(), what, a});
        }
    } tl_;
    PairData D_;
    Stats *S_ = nullptr;
    IterationStream rs_; // sampler + selection/LO streams
    double sample_s_ = 0.0;

    // --- GPU sweeps ---
    // One issuer of single-model sweeps (the estimator thread, or an LO worker during
    // parallel LO steps) with the cache of its last result; `sel` is the
    // selection/LO random stream the issuer draws from.
    struct Lane {
        SweepSlot *slot = nullptr;
        Mt19937 *sel = nullptr;
        Model model;
        bool valid = false;
        double fast = 0.0, bound = 0.0; // the fast sum and its distance bound (lo_sweep_fast)
        bool exact_valid = false;
        double score = 0.0;              // the reference-order sum, once taken
        const double *err = nullptr; // the buffer holding the last result
        std::vector<double> herr;    // host sweeps' errors (3 x n)
        uint64_t count = 0;
        double t[3] = {0, 0, 0}; // -, sweep, - seconds (MADPOSE_SWEEP_TIMING)
    };
    Lane lanes_[kLoLanes]; // lanes_[0]: the estimator thread
    // LO phase seconds (MADPOSE_LO_TIMING): serial prefix, steps phase, LO count, sum of
    // step times, longest step, step-0 time
    // + step 0's non-minimal fit and score, other steps' fit; step 0's first lsq_fit and
    // lsq iterations, the other steps' (mean)
    double lo_t_[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double lo_seg_[3] = {0, 0, 0}; // steps phase: before, during and after the parallel run
    bool lo_parallel_ = true;
    const bool early_hook_ = [] {
        return env_flag("MADPOSE_LO_EARLY_HOOK", true);
    }();

    // LO sweeps run on the issuing thread's core (host/lo_sweep.h): the reference's
    // residual operations and ScoreModel order, bit-identical to the oracle; a lane
    // keeps its last result (LO asks for the same model's score and inliers in turn)
    LoSweepData hsw_;
    // the errors of m (and its fast sum), cached per lane
    const double *sweep(Lane &L, const Model &m) {
        if (L.valid && std::memcmp(&m, &L.model, sizeof(Model)) == 0) return L.err;
        auto t_sw = Clock::now();
        if (L.herr.size() < 3 * (size_t)n_) L.herr.resize(3 * (size_t)n_);
        lo_sweep_fast(P_.C, hsw_, m, L.herr.data(), &L.fast, &L.bound);
        L.err = L.herr.data();
        L.model = m;
        L.valid = true;
        L.exact_valid = false;
        L.count++;
        const double dt = secs(t_sw);
        L.t[1] += dt;
        if (g_prof_on.load(std::memory_order_relaxed)) {
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.sweeps += 1;
            g_prof.sweep_wall_ms += 1e3 * dt;
        }
        return L.err;
    }
    // ScoreModel's reference-order sum of m
    double score(Lane &L, const Model &m) {
        sweep(L, m);
        if (!L.exact_valid) {
            L.score = lo_ordered_score(P_.C, L.err, n_);
            L.exact_valid = true;
        }
        return L.score;
    }
    // Whether m's reference-order score could be below b: false when the fast sum
    // decides it cannot (fast - bound >= b); otherwise the reference-order score in *e
    // (the caller compares it).  UpdateBestModel needs the exact sum only then.
    bool score_below(Lane &L, const Model &m, double b, double *e) {
        sweep(L, m);
        if (!L.exact_valid && L.fast - L.bound >= b) return false;
        *e = score(L, m);
        return true;
    }
    int inliers(Lane &L, const Model &m, const double *thr, std::vector<int> out[3]) {
        const double *e = sweep(L, m);
        // Branch-free compaction: whether a correspondence is an inlier is close to a
        // coin flip along the index, so a conditional push_back mispredicts about every
        // other element (measured on the build host, 3 x 2000 errors at ~50 % inliers:
        // 17.8 us branchy, 5.5 us branch-free scalar).  AVX2: four errors per compare,
        // the lanes below the threshold appended as one 4-index store through a table of
        // the 16 masks (7.1-7.9 -> 3.1 us per 3 x 2000 on the build container).  Same
        // lists (ascending indices).
        int c = 0;
        const __m128i step = _mm_set1_epi32(4);
        for (int t = 0; t < 3; ++t) {
            std::vector<int> &o = out[t];
            o.resize(n_ + 4);
            int *w = o.data(), k = 0, i = 0;
            const double *et = e + (size_t)t * n_;
            const double th = thr[t];
            const __m256d tv = _mm256_set1_pd(th);
            __m128i base = _mm_setzero_si128();
            for (; i + 4 <= n_; i += 4) {
                const int msk = _mm256_movemask_pd(_mm256_cmp_pd(_mm256_loadu_pd(et + i), tv, _CMP_LT_OQ));
                _mm_storeu_si128((__m128i *)(w + k),
                                 _mm_add_epi32(_mm_load_si128((const __m128i *)kCompactLut[msk]), base));
                k += __builtin_popcount((unsigned)msk);
                base = _mm_add_epi32(base, step);
            }
            for (; i < n_; ++i) {
                w[k] = i;
                k += et[i] < th;
            }
            o.resize(k);
            c += k;
        }
        return c;
    }

    static void update_best(double sc, const Model &m, int st, double *best_sc, Model *best, int *best_st) {
        if (sc < *best_sc) {
            *best_sc = sc;
            *best = m;
            *best_st = st;
        }
    }

    uint32_t num_required(int s) const {
        double p_all = 1.0;
        for (int t = 0; t < 3; ++t) p_all *= std::pow(S_->inlier_ratios[t], (double)ss_[s][t]);
        if (p_all <= 0.0) return o_.max_num_iterations_per_solver;
        if (p_all >= 1.0) return o_.min_num_iterations;
        const double p_bad = 1.0 - p_all;
        if (p_bad >= 0.99999999999999) return o_.max_num_iterations_per_solver;
        const double it = std::ceil(std::log(1.0 - o_.success_probability) / std::log(p_bad) + 0.5);
        uint32_t r = std::min((uint32_t)it, o_.max_num_iterations_per_solver);
        return std::max(o_.min_num_iterations, r);
    }

    // UpdateRANSACTerminationCriteria (src/hybrid_ransac.h:351-378)
    void termination(const Model &m, uint32_t *max_per) {
        // after an LO the new best was usually swept last by the LO lane that recorded it:
        // its cached errors give the same inliers as a fresh sweep (the workers are idle
        // between LOs, so their lanes are read here without a race)
        Lane *L = &lanes_[0];
        for (Lane &c : lanes_)
            if (c.valid && std::memcmp(&m, &c.model, sizeof(Model)) == 0) {
                L = &c;
                break;
            }
        S_->best_num_inliers = inliers(*L, m, thr_, S_->inlier_indices);
        for (int t = 0; t < 3; ++t)
            S_->inlier_ratios[t] = n_ > 0 ? (double)S_->inlier_indices[t].size() / (double)n_ : 0.0;
        for (int s = 0; s < 2; ++s) max_per[s] = num_required(s);
    }

    // --- LO (src/hybrid_ransac.h:383-538) ---
    // The batched device LM (kernels/lm_device.h) on the lane's stream instead of the
    // host LM (MADPOSE_DEVICE_LM=1).  The issuing thread sleeps on a blocking-sync event
    // meanwhile, which frees its core for other pairs in flight (estimate_batch).
    bool device_lm_ = false;
    void least_squares_device(Lane &L, const std::vector<int> sample[3], Model *m, bool nonminimal) {
        SweepSlot &sl = *L.slot;
        const int sz[3] = {(int)sample[0].size(), (int)sample[1].size(), (int)sample[2].size()};
        const int64_t nidx = (int64_t)sz[0] + sz[1] + sz[2];
        sl.ensure_lm(nidx);
        constexpr size_t kJob = 0, kOut = 256, kSt = 448, kIdx = 512;
        static_assert(sizeof(LmJob) <= kOut && kOut + sizeof(Model) <= kSt, "LM staging layout");
        const LmJob J = make_lm_job(P_, cfg_, sz, 0, nonminimal, *m);
        std::memcpy(sl.h_lm + kJob, &J, sizeof(J));
        int *hi = (int *)(sl.h_lm + kIdx);
        for (int t = 0, o = 0; t < 3; ++t) {
            std::memcpy(hi + o, sample[t].data(), sizeof(int) * sz[t]);
            o += sz[t];
        }
        MP_HIP(hipMemcpyAsync(sl.d_lm, sl.h_lm, kIdx + sizeof(int) * (size_t)nidx, hipMemcpyHostToDevice, sl.stream));
        MP_HIP(launch_lm_batch(sl.stream, D_, P_.C, (const LmJob *)(sl.d_lm + kJob), 1, (const int *)(sl.d_lm + kIdx),
                               (Model *)(sl.d_lm + kOut), (int *)(sl.d_lm + kSt)));
        MP_HIP(hipMemcpyAsync(sl.h_lm + kOut, sl.d_lm + kOut, kIdx - kOut, hipMemcpyDeviceToHost, sl.stream));
        MP_HIP(hipEventRecord(sl.lm_done, sl.stream));
        MP_HIP(hipEventSynchronize(sl.lm_done));
        std::memcpy(m, sl.h_lm + kOut, sizeof(Model));
    }

    void least_squares(Lane &L, const std::vector<int> sample[3], Model *m, bool nonminimal) {
        const int kmd = variant_ == kCal ? 3 : 4;
        if (((int)sample[0].size() < kmd && (int)sample[1].size() < kmd) || (int)sample[2].size() < min_sample_size_)
            return;
        if (device_lm_) {
            auto t_lm = Clock::now();
            least_squares_device(L, sample, m, nonminimal);
            if (g_prof_on.load(std::memory_order_relaxed)) {
                std::lock_guard<std::mutex> lk(g_prof_mu);
                g_prof.lm_calls += 1;
                g_prof.lm_wall_ms += 1e3 * secs(t_lm);
            }
            return;
        }
        LMSettings S;
        S.use_reproj = cfg_.lo_type != 1;
        S.use_sampson = cfg_.lo_type != 2;
        // use_shift is forwarded by the calibrated estimator (NonMinimalSolver and
        // LeastSquares) and by the shared-focal NonMinimalSolver only.
        S.use_shift = (variant_ == kCal || (variant_ == kSF && nonminimal)) ? cfg_.use_shift : true;
        S.min_depth_constraint = cfg_.min_depth_constraint;
        if (P_.C.scale_only) { // HybridPoseOptimizerScaleOnly: offsets constant, unbounded
            S.use_shift = false;
            S.min_depth_constraint = false;
        }
        S.w_sampson = variant_ == kCal ? std::sqrt(P_.H.sampson_squared_weight) /
                                             (1.0 / (P_.C.K0[0] + P_.C.K0[4]) + 1.0 / (P_.C.K1[0] + P_.C.K1[4]))
                                       : std::sqrt(P_.H.sampson_squared_weight);
        S.ftol = cfg_.ftol;
        S.gtol = cfg_.gtol;
        S.ptol = cfg_.ptol;
        S.max_iter = (int)cfg_.max_iter;
        S.nonmonotonic = cfg_.nonmonotonic;
        auto t_lm = Clock::now();
        lm_refine(P_.H, sample, S, m);
        if (lo_timing_) {
            const size_t nb = (S.use_reproj ? sample[0].size() + sample[1].size() : 0) +
                              (S.use_sampson ? sample[2].size() : 0);
            if (nb >= kBigLM) {
                std::lock_guard<std::mutex> lk(lm_stat_mu_);
                lm_stat_[0] += 1.0;
                lm_stat_[1] += lm_last_evals;
                lm_stat_[2] += secs(t_lm);
                lm_stat_[3] += (double)nb;
            }
        }
        if (g_prof_on.load(std::memory_order_relaxed)) {
            const double dt = secs(t_lm);
            const size_t nb = (S.use_reproj ? sample[0].size() + sample[1].size() : 0) +
                              (S.use_sampson ? sample[2].size() : 0);
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.lm_calls += 1;
            g_prof.lm_wall_ms += 1e3 * dt;
            g_prof.lm_blocks += nb;
            if (nb >= kBigLM) {
                g_prof.lm_big_calls += 1;
                g_prof.lm_big_wall_ms += 1e3 * dt;
            }
        }
    }

    // all: indices idx + t * n (t < 3, shuffled, so the type is random along the list);
    // branch-free like inliers()
    static void split(const std::vector<int> &all, int n, std::vector<int> out[3]) {
        const size_t m = all.size();
        for (int t = 0; t < 3; ++t) out[t].resize(m);
        int *w0 = out[0].data(), *w1 = out[1].data(), *w2 = out[2].data();
        int k0 = 0, k1 = 0, k2 = 0;
        for (size_t i = 0; i < m; ++i) {
            const int idx = all[i];
            const int t = (idx >= n) + (idx >= 2 * n);
            const int v = idx - t * n;
            w0[k0] = v;
            w1[k1] = v;
            w2[k2] = v;
            k0 += t == 0;
            k1 += t == 1;
            k2 += t == 2;
        }
        out[0].resize(k0);
        out[1].resize(k1);
        out[2].resize(k2);
    }
    static void shuffle_resize(Mt19937 &sel, int k, std::vector<int> *v) {
        const int n = (int)v->size();
        if (n <= k) return;
        for (int i = 0; i < k; ++i) std::swap((*v)[i], (*v)[uniform_int(sel, i, n - 1)]);
        v->resize(k);
    }
    // draws of one lsq_fit when every data type has enough inliers (the usual case)
    int lsq_fit_draws(int st) const {
        int k = 0;
        for (int t = 0; t < 3; ++t) k += ss_[st][t] * o_.min_sample_multiplicator;
        return k * o_.min_sample_multiplicator;
    }

    void lsq_fit(Lane &L, const double *thr, int st, Model *m, bool use_all) {
        std::vector<int> inl[3];
        inliers(L, *m, thr, inl);
        int k[3];
        for (int t = 0; t < 3; ++t) {
            if ((int)inl[t].size() < ss_[st][t]) return;
            k[t] = std::min(ss_[st][t] * o_.min_sample_multiplicator, (int)inl[t].size());
        }
        if (use_all) {
            least_squares(L, inl, m, false);
            return;
        }
        const int total = (k[0] + k[1] + k[2]) * o_.min_sample_multiplicator;
        std::vector<int> all;
        all.reserve(inl[0].size() + inl[1].size() + inl[2].size());
        for (int t = 0; t < 3; ++t)
            for (int idx : inl[t]) all.push_back(idx + t * n_);
        shuffle_resize(*L.sel, total, &all);
        std::vector<int> smp[3];
        split(all, n_, smp);
        least_squares(L, smp, m, false);
    }

    // The non-minimal sample of an LO step is unusable (NonMinimalSolver returns 0,
    // or Solve() sees no residuals): the step is skipped without drawing.
    bool step_skipped(const std::vector<int> &sample_all) const {
        // (the sizes split() would give, counted without building the lists: this runs
        // on the estimator thread before the parallel steps start)
        int cnt[3] = {0, 0, 0};
        for (const int idx : sample_all) cnt[(idx >= n_) + (idx >= 2 * n_)]++;
        const int kmd = variant_ == kCal ? 3 : 4;
        if ((cnt[0] < kmd && cnt[1] < kmd) || cnt[2] < min_sample_size_) return true;
        const size_t nres = (cfg_.lo_type != 1 ? (size_t)cnt[0] + cnt[1] : 0) + (cfg_.lo_type != 2 ? (size_t)cnt[2] : 0);
        return nres == 0;
    }
    struct StepOut {
        std::vector<std::pair<double, Model>> updates; // the step's update_best calls, in order
        Mt19937 sel;                                   // LO stream after the step
        double nonmin_s = 0.0, score_s = 0.0;          // MADPOSE_LO_TIMING: non-minimal fit, its score,
        double lsq_s = 0.0, iter_s = 0.0;              // the first lsq_fit, the lsq iterations
    };
    // One LO step (the loop body of src/hybrid_ransac.h:435-470) from m_init on the
    // non-minimal sample `sample_all`, drawing from *L.sel.
    // The step's update_best calls are applied after all steps, in step order, so a
    // score can update the best only if it is below b0 (the best when the steps start:
    // later bests are lower) and below every score this step recorded before it; scores
    // the fast sum puts at or above that are not recorded (score_below).
    void lo_step(Lane &L, int st, const std::vector<int> &sample_all, const Model &m_init, const double *thr,
                 const double *upd, double b0, StepOut &out) {
        out.updates.clear();
        if (step_skipped(sample_all)) return;
        double b = b0;
        auto record = [&](const Model &mm) {
            double e;
            if (score_below(L, mm, b, &e)) {
                out.updates.emplace_back(e, mm);
                b = std::min(b, e);
            }
        };
        Model m = m_init;
        std::vector<int> smp[3];
        split(sample_all, n_, smp);
        auto t_nm = Clock::now();
        least_squares(L, smp, &m, true);
        out.nonmin_s = secs(t_nm);
        auto t_sc = Clock::now();
        record(m);
        out.score_s = secs(t_sc);
        auto t_l = Clock::now();
        lsq_fit(L, thr_, st, &m, false);
        out.lsq_s = secs(t_l);
        double cur[3] = {thr[0], thr[1], thr[2]};
        auto t_it = Clock::now();
        for (int i = 0; i < o_.num_lsq_iterations; ++i) {
            lsq_fit(L, cur, st, &m, false);
            record(m);
            for (int t = 0; t < 3; ++t) cur[t] -= upd[t];
        }
        out.iter_s = secs(t_it);
    }

    // LocalOptimization (src/hybrid_ransac.h:383-470).  The steps depend on each
    // other only through the LO random stream, and each step draws a predictable
    // number of values (lsq_fit_draws per lsq_fit) unless an lsq_fit finds too few
    // inliers or a draw is rejected.  So the steps run concurrently on kLoLanes
    // threads from the stream positions they would start at; afterwards every
    // step's end position is checked against the next step's start, steps after a
    // mismatch are recomputed in order, and the steps' update_best calls are applied
    // in step order -- the result is the serial one in every case.
    // predicted(sel): called once the LO stream's end state is predicted (parallel
    // steps), before the steps run -- the estimator speculates the next batch on it.
    void local_opt(int st, Model *best_min, double *best_min_score, int *best_st,
                   const std::function<void(const Mt19937 &)> &predicted = nullptr) {
        auto t0 = Clock::now();
        Lane &L0 = lanes_[0];
        double thr[3], upd[3];
        for (int t = 0; t < 3; ++t) {
            upd[t] = (o_.threshold_multiplier - 1.0) * thr_[t] / (int)(o_.num_lsq_iterations - 1);
            thr[t] = thr_[t] * o_.threshold_multiplier;
        }
        // Early hook (MADPOSE_LO_EARLY_HOOK=0 turns it off): the stream's end is predicted
        // before the serial prefix, so the speculative batch is on the GPU while the prefix
        // runs.  The prefix's shuffle draws k_nonmin values when the base inlier set is
        // larger -- k_nonmin = max(non_min_sample_size, min(min_sample_size x multiplier,
        // |base| / 2)) is that constant whenever |base| / 2 reaches the product (always for
        // the default options: 35 >= 15) -- and every step draws per_step unless it is
        // skipped.  Any other outcome ends the LO elsewhere and the speculation is
        // discarded (the caller compares the draw counts), as for the late prediction.
        bool hooked = false;
        const int R_steps = o_.num_lo_steps;
        if (predicted && early_hook_ && lo_parallel_ && R_steps > 1) {
            const uint64_t per_step = (uint64_t)(1 + o_.num_lsq_iterations) * (uint64_t)lsq_fit_draws(st);
            const int k_pred = std::max(non_min_sample_size_, min_sample_size_ * o_.non_min_sample_multiplier);
            Mt19937 e = rs_.sel;
            e.discard((uint64_t)k_pred + (uint64_t)R_steps * per_step);
            predicted(e);
            hooked = true;
        }
        Model m_init = *best_min;
        lsq_fit(L0, thr, st, &m_init, true);
        double sc;
        if (score_below(L0, m_init, *best_min_score, &sc)) update_best(sc, m_init, st, best_min_score, best_min, best_st);
        const double b0 = *best_min_score; // (the steps' scores are decided against it, lo_step)
        std::vector<int> base[3];
        inliers(L0, m_init, thr_, base);
        std::vector<int> base_all;
        for (int t = 0; t < 3; ++t)
            for (int idx : base[t]) base_all.push_back(idx + t * n_);
        const int k_nonmin = std::max(non_min_sample_size_,
                                      std::min(min_sample_size_ * o_.non_min_sample_multiplier, (int)base_all.size() / 2));
        const int R = o_.num_lo_steps;
        lo_t_[0] += secs(t0); // serial prefix: initial fit, score, base inliers
        tl_.mark("lo_prefix_end", (long)base_all.size());
        auto t_steps = Clock::now();
        if (R > 0) {
            // step 0 solves on base_all as it is and then shuffles it down to
            // k_nonmin; later steps shuffle nothing (it is that size already) and all
            // solve on the shuffled sample (:439-440)
            const std::vector<int> sample0 = base_all;
            shuffle_resize(rs_.sel, k_nonmin, &base_all);
            const std::vector<int> &sample1 = base_all;
            std::vector<StepOut> outs(R);
            int first_serial = 0; // steps [first_serial, R) still to run in order
            Mt19937 sel = rs_.sel;
            if (lo_parallel_ && R > 1) {
                std::vector<uint64_t> start(R);
                uint64_t pos = sel.draws();
                const uint64_t per_step = (uint64_t)(1 + o_.num_lsq_iterations) * (uint64_t)lsq_fit_draws(st);
                const bool skip0 = step_skipped(sample0), skip1 = R > 1 && step_skipped(sample1);
                for (int r = 0; r < R; ++r) {
                    start[r] = pos;
                    if (!(r == 0 ? skip0 : skip1)) pos += per_step;
                }
                const Mt19937 base_sel = sel;
                // the speculation hook runs as job 1, beside the steps: step 0 (the
                // longest, on all base inliers) starts at once, and the lane that takes
                // the hook takes a short step after it (the hook may wait for the
                // sampler thread to finish launching a continuation it cancels)
                Mt19937 end = base_sel;
                const bool hook_job = predicted && !hooked && X_.lo_workers->lanes() > 1;
                if (predicted && !hooked) {
                    end.discard(pos - base_sel.draws());
                    if (!hook_job) predicted(end);
                }
                std::vector<double> step_s(R, 0.0);
                const auto t_run = Clock::now();
                lo_seg_[0] += std::chrono::duration<double>(t_run - t_steps).count();
                X_.lo_workers->run(R + (hook_job ? 1 : 0), [&](int job, int lane) {
                    if (hook_job && job == 1) {
                        auto th = Clock::now();
                        if (lane != 0) MP_HIP(hipSetDevice(X_.device));
                        predicted(end);
                        lo_seg_[2] += secs(th);
                        return;
                    }
                    const int r = hook_job && job > 1 ? job - 1 : job;
                    auto ts = Clock::now();
                    if (lane != 0) MP_HIP(hipSetDevice(X_.device));
                    Mt19937 my = base_sel;
                    my.discard(start[r] - base_sel.draws());
                    Lane &L = lanes_[lane];
                    L.sel = &my;
                    lo_step(L, st, r == 0 ? sample0 : sample1, m_init, thr, upd, b0, outs[r]);
                    L.sel = lane == 0 ? &rs_.sel : nullptr;
                    outs[r].sel = my;
                    step_s[r] = secs(ts);
                });
                lo_seg_[1] += secs(t_run);
                for (int r = 0; r < R; ++r) {
                    lo_t_[3] += step_s[r];
                    lo_t_[4] = std::max(lo_t_[4], step_s[r]);
                }
                lo_t_[5] += step_s[0];
                lo_t_[6] += outs[0].nonmin_s;
                lo_t_[7] += outs[0].score_s;
                for (int r = 1; r < R; ++r) lo_t_[8] += outs[r].nonmin_s / (R - 1);
                lo_t_[9] += outs[0].lsq_s;
                lo_t_[10] += outs[0].iter_s;
                for (int r = 1; r < R; ++r) {
                    lo_t_[11] += outs[r].lsq_s / (R - 1);
                    lo_t_[12] += outs[r].iter_s / (R - 1);
                }
                // steps 0..r are right while each one ended where the next one started
                first_serial = R;
                for (int r = 0; r + 1 < R; ++r)
                    if (outs[r].sel.draws() != start[r + 1]) {
                        first_serial = r + 1;
                        break;
                    }
                sel = outs[first_serial - 1].sel;
                if (trace_ && first_serial < R)
                    std::fprintf(stderr, "[engine] LO step %d started off its predicted draw; recomputing\n",
                                 first_serial);
            }
            lo_t_[13] += R - first_serial; // steps recomputed in order
            for (int r = first_serial; r < R; ++r) {
                L0.sel = &sel;
                lo_step(L0, st, r == 0 ? sample0 : sample1, m_init, thr, upd, b0, outs[r]);
                L0.sel = &rs_.sel;
            }
            rs_.sel = sel;
            for (int r = 0; r < R; ++r)
                for (const auto &u : outs[r].updates) update_best(u.first, u.second, st, best_min_score, best_min, best_st);
        }
        lo_t_[1] += secs(t_steps);
        lo_t_[2] += 1.0;
        S_->seconds_lo += secs(t0);
    }

    // --- minimal-sample batches (host) ---
    // Batches drawn on this thread (at the start, after LO or a cut batch) are sized so
    // drawing them costs about one batch round trip on the GPU: cheap solvers get short
    // synchronous batches (the worker draws the long ones), expensive ones long.
    double draw_s_per_it_ = 40e-9, batch_s_ = 1e-3; // running estimates
    uint32_t sync_batch(uint32_t want) const {
        const double b = batch_s_ / std::max(draw_s_per_it_, 1e-9);
        return std::min<uint32_t>(want, (uint32_t)std::max<double>(min_batch_, std::min<double>(b, 1e9)));
    }
    int *slot_ptr(int slot) const { return X_.h_samples + (size_t)slot * 9 * max_batch_; }
    // slot_ptr for a draw or an upload of B iterations, bounds-checked on the host: slot s
    // spans [9 s max_batch_, 9 (s + 1) max_batch_) of the 2 x 9 cap_b ints of h_samples
    // (every draw into and upload from a slot is range-checked)
    int *slot_for(int slot, uint32_t B) const {
        if (slot < 0 || slot > 1 || B > (uint32_t)max_batch_ || max_batch_ > X_.cap_b || !X_.h_samples)
            throw std::logic_error("sample slot out of range: slot " + std::to_string(slot) + ", B " +
                                   std::to_string(B) + ", max_batch " + std::to_string(max_batch_) + ", cap_b " +
                                   std::to_string(X_.cap_b));
        return slot_ptr(slot);
    }
    void generate(Batch &g, uint32_t B, int slot) {
        auto t0 = Clock::now();
        draw_batch(rs_, g, B, slot, slot_for(slot, B), nullptr, sampler_mode());
        sample_s_ += secs(t0);
    }
    // both streams to the end of iteration j of batch g
    void rewind(const Batch &g, uint32_t j) {
        auto t0 = Clock::now();
        const uint32_t k = j / kSnap;
        rs_ = g.snaps[k];
        int scratch[8];
        for (uint32_t r = k * kSnap; r <= j; ++r) rs_.next(scratch);
        sample_s_ += secs(t0);
    }

    // Solves and scores batch g on the GPU (asynchronous, X_.stream): sample upload,
    // MD solver on the side stream, the point-solver stages, score_batch, and the
    // per-iteration best scores / slots / model counts back to pinned host memory.
    // best: best_min_model_score when the batch starts (the scoring's early exit).
    bool batch_prof_[2] = {false, false};
    double launch_s_ = 0.0; // main-thread time in launch_batch (MADPOSE_LO_TIMING)
    // early continuation: off by default (MADPOSE_EARLY_CONT=1: on while this estimator
    // is alone on its device, =2: always).  With 8 shared-focal pairs in flight the
    // discarded continuations took GPU time from the other pairs (ScanNet stand-in 747
    // -> 1064 pairs/s without them, profiles/r04/scab/); alone, an LO that cancels the
    // continuation waits for the sampler thread to finish launching it (the speculation
    // hook 31-48 us instead of 4 us, the LO steps phase 221-233 vs 180-194 us, cal 5.90-
    // 5.99 vs 5.80-5.86 ms, profiles/r04/hook2/)
    // =3: continuations of at least kEarlyMinBatch iterations while alone on the device
    // (the growth phase, where new bests are rare): each slot has its own stream, so the
    // continuation's solvers run while this batch is scored.  Its gating is best-effort
    // (ADVICE r05): the continuation waits only for the previous batch's solve, so both
    // score kernels can run at once against the one record word, and the newer epoch's
    // atomicMin can replace the older batch's record -- the older batch's workgroups then
    // stop skipping and the continuation is no longer cancelled by it.  Results do not
    // change (the host walks and discards as always); a discarded continuation merely
    // costs its full GPU time.  (On one stream, round 5's
    // first form, it measured slower: cal 5.62 -> 5.86 ms per pair, profiles/r05/r5o.)
    const int early_mode_ = [] {
        return (int)env_int("MADPOSE_EARLY_CONT", 0, 0, 3);
    }();
    static constexpr uint32_t kEarlyMinBatch = 4096;
    bool early_now(uint32_t Bn) const {
        return early_mode_ == 2 || (early_mode_ == 1 && active_runs(X_.device) <= 1) ||
               (early_mode_ == 3 && Bn >= kEarlyMinBatch && active_runs(X_.device) <= 1);
    }
    int launch_n_ = 0;
    // big LM solves (>= kBigLM blocks) under MADPOSE_LO_TIMING: count, evaluations,
    // seconds, blocks
    const bool lo_timing_ = std::getenv("MADPOSE_LO_TIMING") != nullptr;
    std::mutex lm_stat_mu_;
    double lm_stat_[4] = {0, 0, 0, 0};
    // the fused MD + 5pt launches up to this batch size (MADPOSE_SOLVE_FUSE_MAX; default:
    // every batch).  Round 5's one-stage fused kernel (216 VGPRs, two waves per SIMD) cost
    // the 5pt root stage its third wave on big batches (cal 5.62 always fused -> 5.46 ms
    // up to 8192, profiles/r05/r5o); the two-stage form (md_setup_pt5 + md_root_tail5)
    // runs the big batches faster than the MD side stream beside the point chain: cal
    // gpu_solve 2.10 -> 2.02 ms, 3.99 -> 3.90 ms per pair (5 same-box A/B pairs,
    // profiles/r06/fuse_all)
    const int64_t fuse_max_ = [] {
        return (int64_t)env_int("MADPOSE_SOLVE_FUSE_MAX", 1ll << 40, 0, 1ll << 40);
    }();

    // cut_on_record: the batch lies at or past lo_starting_iterations, so its first new
    // best runs LO and cuts it; score_batch then skips the iterations behind a record.
    // gate_prev: the batch is launched before the previous one's results were read (an
    // early continuation); its kernels leave at once if that batch published a record
    // (kernels.h batch_cancelled), i.e. if the host is bound to discard this one.
    void launch_batch(const Batch &g, double best, bool cut_on_record, const BatchBufs *gate_prev = nullptr) {
        const uint32_t B = g.B;
        const int nmd = g.nmd, npt = g.npt;
        BatchBufs &Q = X_.bb[g.slot];
        const BatchBufs &O = X_.bb[g.slot ^ 1];
        hipStream_t s = Q.stream;
        const bool prof = g_prof_on.load(std::memory_order_relaxed);
        batch_prof_[g.slot] = prof;
        PairData D = D_;
        if (gate_prev) {
            D.gate = X_.d_recword;
            D.gate_hi = gate_prev->epoch_hi;
        }
        // one upload: samples, then the MD list and the (descending) point list
        MP_HIP(hipMemcpyAsync(Q.d_samples, slot_for(g.slot, B), sizeof(int) * 9 * (size_t)B, hipMemcpyHostToDevice, s));
        tl_.mark("  h2d");
        MP_HIP(hipEventRecord(Q.ev_h2d, s));
        Q.h2d_pending = true;
        const int *d_md_list = Q.d_samples + 8 * (size_t)B, *d_pt_list = d_md_list + nmd;
        // (the other slot's batch may still be solving: the solvers' workspace is shared)
        MP_HIP(hipStreamWaitEvent(s, O.ev_solved, 0));
        if (prof) MP_HIP(hipEventRecord(Q.ev[0], s));
        // MD iterations on the side stream, point iterations on the main one (they
        // write disjoint model slots); scoring waits for both -- or, calibrated, both in
        // one launch on the main stream (launch_solve_fused)
        const PtWorkspace W{X_.d_pt_cand, X_.d_pt_ncand, X_.d_pt_slots, X_.d_pt_valid, X_.d_pt_pen,
                            X_.d_md_ws,   X_.d_md_nr,   X_.cap_b};
        const bool fused = solve_fusable(P_.C) && (int64_t)B <= fuse_max_;
        if (fused) {
            MP_HIP(launch_solve_fused(s, D, P_.C, d_md_list, nmd, d_pt_list, npt, Q.d_samples, W, Q.d_models,
                                      Q.d_recs, Q.d_counts, maxm_));
            tl_.mark("  solve_launched");
        } else {
            if (nmd > 0) {
                MP_HIP(hipEventRecord(Q.ev_fork, s));
                MP_HIP(hipStreamWaitEvent(X_.md_stream, Q.ev_fork, 0));
                MP_HIP(launch_md_solve_staged(X_.md_stream, D, P_.C, d_md_list, nmd, Q.d_samples, W, Q.d_models,
                                              Q.d_recs, Q.d_counts, maxm_));
                MP_HIP(hipEventRecord(Q.ev_join, X_.md_stream));
            }
            MP_HIP(launch_pt_solve(s, D, P_.C, d_pt_list, npt, Q.d_samples, W, Q.d_models, Q.d_recs, Q.d_counts,
                                   maxm_));
            if (nmd > 0) MP_HIP(hipStreamWaitEvent(s, Q.ev_join, 0));
        }
        MP_HIP(hipEventRecord(Q.ev_solved, s));
        if (prof) MP_HIP(hipEventRecord(Q.ev[1], s));
        const unsigned epoch_hi = ~(++X_.epoch);
        Q.epoch_hi = epoch_hi;
        MP_HIP(launch_score_batch(s, D, P_.C, Q.d_recs, Q.d_counts, (int)B, maxm_, Q.d_scores, Q.d_res, best,
                                  prof ? Q.d_work : nullptr, cut_on_record ? X_.d_recword : nullptr, epoch_hi,
                                  Q.d_models, Q.d_recmodel, Q.d_flags8, Q.d_cand));
        tl_.mark("  score_launched");
        if (prof) MP_HIP(hipEventRecord(Q.ev[2], s));
        MP_HIP(hipMemcpyAsync(Q.h_flags8, Q.d_flags8, (size_t)B, hipMemcpyDeviceToHost, s));
        if (prof) MP_HIP(hipMemcpyAsync(Q.h_work, Q.d_work, sizeof(int) * B, hipMemcpyDeviceToHost, s));
        MP_HIP(hipEventRecord(Q.ev_done, s));
    }
    // every batch launched from this run has finished (both slots' streams and the MD
    // side stream)
    void drain_batches() {
        for (const BatchBufs &q : X_.bb) MP_HIP(hipStreamSynchronize(q.stream));
        MP_HIP(hipStreamSynchronize(X_.md_stream));
    }
    // before host sample slot `slot` is redrawn: the last batch launched from it must
    // have been copied to the device (an early continuation may still be queued)
    void slot_free(int slot) {
        BatchBufs &Q = X_.bb[slot];
        if (Q.h2d_pending) {
            MP_HIP(hipEventSynchronize(Q.ev_h2d));
            Q.h2d_pending = false;
        }
    }

    // Reference-order score of a model (host/lo_sweep.h), on lane 0: the LO that follows
    // a new best starts with a sweep of the same model and finds it cached.
    double exact_score(const Model &m) { return score(lanes_[0], m); }

    // Iteration j of the last batch could hold a new best but it is not certain which of
    // its models wins in the reference order: its best's interval [S - T, S + T] reaches
    // another model's (kSlotAmbiguous), best_min_score lies inside it, or the iteration
    // is uncertain (a flagged correspondence: no margin holds, every model is a
    // contender).  Re-score the contenders in the reference's order and take the first
    // minimum (GetBestEstimatedModelId, src/hybrid_ransac.h:245-263); a model whose lower
    // bound S - T exceeds the smallest upper bound of the iteration cannot be the
    // reference's winner.  Rare (tests/test_ties_gpu.py forces it).
    void resolve_tie(const BatchBufs &Q, uint32_t j, Model *out, double *out_score) {
        const int nm = Q.h_cand[j].count;
        const bool uncertain = (Q.h_cand[j].slot & kSlotUncertain) != 0;
        std::vector<double> dsc(nm);
        std::vector<Model> ms(nm);
        std::vector<ScoreRec> rc(nm);
        // (the batch is complete; the main stream may already hold the next one)
        MP_HIP(hipMemcpyAsync(dsc.data(), Q.d_scores + (size_t)j * maxm_, sizeof(double) * nm,
                              hipMemcpyDeviceToHost, X_.copy_stream));
        MP_HIP(hipMemcpyAsync(ms.data(), Q.d_models + (size_t)j * maxm_, sizeof(Model) * nm, hipMemcpyDeviceToHost,
                              X_.copy_stream));
        MP_HIP(hipMemcpyAsync(rc.data(), Q.d_recs + (size_t)j * maxm_, sizeof(ScoreRec) * nm, hipMemcpyDeviceToHost,
                              X_.copy_stream));
        MP_HIP(hipStreamSynchronize(X_.copy_stream));
        double hi_min = kMax; // the smallest upper bound of a model's reference-order score
        for (int m = 0; m < nm; ++m)
            if (dsc[m] < kMax) hi_min = std::min(hi_min, dsc[m] + rc[m].tie);
        *out_score = kMax;
        for (int m = 0; m < nm; ++m) {
            // (a model the exit killed reports DBL_MAX: its reference sum reached the
            // pre-batch best, it cannot win)
            if (!uncertain && (!(dsc[m] < kMax) || dsc[m] - rc[m].tie > hi_min)) continue;
            const double e = exact_score(ms[m]);
            if (e < *out_score) { // strict '<': the first minimum wins
                *out_score = e;
                *out = ms[m];
            }
        }
        ++tie_checks_;
    }

    // the model of a new best: score_batch wrote it to the mapped record slot of its
    // iteration (the batch's stream has been synchronized)
    Model fetch_model(const BatchBufs &Q, int b) { return Q.h_recmodel[b]; }
};

void Run::run(Model *best, Stats *S) {
    auto t_start = Clock::now();
    const char *dump_path = std::getenv("MADPOSE_COUNT_DUMP");
    std::unique_ptr<FILE, int (*)(FILE *)> dump(dump_path ? std::fopen(dump_path, "w") : nullptr, &std::fclose);
    count_dump_ = dump.get();
    const char *mdump_path = std::getenv("MADPOSE_MODEL_DUMP");
    std::unique_ptr<FILE, int (*)(FILE *)> mdump(mdump_path ? std::fopen(mdump_path, "wb") : nullptr, &std::fclose);
    model_dump_ = mdump.get();
    {
        static std::atomic<long> runs{0};
        const long r = runs.fetch_add(1);
        const char *e = std::getenv("MADPOSE_TIMELINE");
        long lo = -1, hi = -1; // "k" or "k-m"
        if (e) {
            int used = 0;
            const int k = std::sscanf(e, "%ld%n-%ld%n", &lo, &used, &hi, &used);
            if (k < 1 || e[used] != '\0' || lo < 0 || (k == 2 && hi < lo)) env_reject("MADPOSE_TIMELINE", e, "expected k or k-m");
            if (k < 2) hi = lo;
        }
        tl_.on = e && r >= lo && r <= hi;
        tl_.run = r;
        tl_.t0 = t_start;
    }
    S_ = S;
    *S = Stats();
    S->best_model_score = kMax;
    std::memset(best, 0, sizeof(Model));
    best->scale = 1.0;
    best->focal0 = best->focal1 = 1.0;
    double *prior = rs_.prior;
    if (cfg_.solver_type == 1) prior[0] = 0.0;
    if (cfg_.solver_type == 2) prior[1] = 0.0;
    for (int s = 0; s < 2; ++s)
        for (int t = 0; t < 3; ++t) {
            rs_.ss[s][t] = ss_[s][t];
            if (ss_[s][t] > n_) prior[s] = 0.0;
        }
    if (prior[0] <= 0.0 && prior[1] <= 0.0) { // VerifyData failed
        S->seconds_total = secs(t_start);
        return;
    }
    X_.ensure(n_, max_batch_, maxm_);
    if (!X_.sampler) X_.sampler.reset(new Sampler());
    lanes_[0].slot = &X_.sweep_slot[0];
    lanes_[0].sel = &rs_.sel;
    {
        lo_parallel_ = env_flag("MADPOSE_LO_PARALLEL", true) && o_.num_lo_steps > 1;
        device_lm_ = env_flag("MADPOSE_DEVICE_LM", false);
    }
    if (lo_parallel_) {
        const int nl = lo_lanes_setting();
        if (!X_.lo_workers || X_.lo_workers->lanes() != nl) X_.lo_workers.reset(new LoWorkers(nl, X_.device));
        for (int l = 1; l < nl; ++l) lanes_[l].slot = &X_.sweep_slot[l];
    }
    upload_pair(X_, P_, &D_);
    lo_sweep_prepare(P_.C, P_.H.x0.data(), P_.H.x1.data(), P_.H.d0.data(), P_.H.d1.data(), &hsw_);
    rs_.n = n_;
    rs_.seed(o_.random_seed);

    const uint32_t max_total = std::max(o_.max_num_iterations, o_.min_num_iterations);
    uint32_t max_per[2];
    max_per[0] = max_per[1] = std::max(o_.max_num_iterations_per_solver, o_.min_num_iterations);
    const uint32_t lo_start = (uint32_t)o_.lo_starting_iterations;
    Model best_min;
    std::memset(&best_min, 0, sizeof(best_min));
    double best_min_score = kMax;

    uint32_t it = 0;
    bool done = false;
    int bcur = min_batch_;
    // batch size at position `at`: the solver kernels are latency-bound (cost ~flat
    // up to tens of thousands of samples) and new bests -- the only thing that cuts
    // a batch -- thin out like records of an iid sequence, so speculate on a window
    // proportional to the position in the stream; batches stop at lo_start.
    auto batch_size = [&](uint32_t at, uint32_t want) {
        uint32_t B = std::min<uint32_t>(want, max_total - at);
        if (at < lo_start) B = std::min<uint32_t>(B, lo_start - at);
        // the loop stops once a solver type reaches its (termination-adjusted) cap:
        // iterations past the expected stop would be scored for nothing.  Expected
        // stop of type st from here: its remaining count over its selection share
        // (+10 % and a few iterations of slack; a short batch only costs a round trip).
        const double ps = prior[0] + prior[1];
        double cap = 1e18;
        for (int st = 0; st < 2; ++st) {
            if (prior[st] <= 0.0) continue;
            const double share = prior[st] / ps;
            const double left = (double)max_per[st] - (double)S->num_iterations_per_solver[st] -
                                share * (double)(at > it ? at - it : 0);
            cap = std::min(cap, std::max(0.0, left) / share * 1.1 + 32.0);
        }
        if (cap < (double)B) B = std::max<uint32_t>(1, (uint32_t)cap);
        return B;
    };
    // speculation window at `at`: growth_ x at iterations, clamped to [min, max]
    auto grow = [&](uint32_t at) {
        return (uint32_t)std::min<double>((double)max_batch_, std::max<double>((double)min_batch_, growth_ * at));
    };
    Batch gen[2];
    // the worker may be drawing into gen[] when an exception unwinds this frame
    struct CancelOnExit {
        Sampler *s;
        ~CancelOnExit() { s->cancel(); }
    } cancel_on_exit{X_.sampler.get()};
    int cur = 0;
    bool have_next = false; // gen[cur] already holds the batch starting at `it`
    bool launched = false;  // ... and it is already on the GPU (post-LO speculation)
    // Post-LO speculation (MADPOSE_LO_SPECULATE=0 disables): the batch after an LO
    // depends on the LO only through the selection stream's end state, which the
    // parallel LO predicts before its steps run.  The sampler draws that batch from the
    // predicted state and launches it while the steps run; it is kept if the LO ends
    // exactly there (else discarded), so results never depend on the speculation.
    const bool speculate = [] {
        return env_flag("MADPOSE_LO_SPECULATE", true);
    }();
    // Chained speculation (MADPOSE_LO_CHAIN=0 disables): the sampler job of the post-LO
    // batch (at `at`, Bs iterations, in `slot`) also draws the batch after it into the
    // other slot, whose batch -- the one that led to the LO -- is spent; if the
    // speculative batch comes next and leads to no LO, that one is next and is already
    // drawn when the host has read the speculative batch.
    const bool chain_on = [] {
        return env_flag("MADPOSE_LO_CHAIN", true);
    }();
    // gen[cur ^ 1] holds (or the sampler is still drawing, until chained()) the batch
    // of chain_B iterations from chain_at on
    bool chain_ready = false;
    uint32_t chain_at = 0, chain_B = 0;
    // MADPOSE_LO_CHAIN_LAUNCH=1: the job also launches the chained batch, behind the
    // speculative batch (the GPU otherwise idles for the rest of the LO), bound by the
    // pre-LO best and gated on the speculative batch's record word (kernels.h
    // batch_cancelled) like an early continuation; when the host discards it, the next
    // batch in its slot follows it on the slot's stream.  Off by default: cal 4.28 ->
    // 4.24 ms, sf 9.72 -> 9.93 ms (its discarded batches overlap the next scoring,
    // profiles/r05/chain_launch).
    const bool chain_launch = [] {
        return env_flag("MADPOSE_LO_CHAIN_LAUNCH", false);
    }();
    auto make_chain = [&](uint32_t at, uint32_t Bs, int slot, double bound, Sampler::Chain *ch, uint32_t *ch_at,
                          uint32_t *ch_B) {
        const uint32_t at2 = at + Bs;
        if (!chain_on || early_mode_ != 0 || at2 >= max_total || at2 == lo_start) return false;
        const uint32_t B2 = batch_size(at2, grow(at2));
        if (B2 == 0) return false;
        slot_free(slot ^ 1);
        Batch *g2 = &gen[slot ^ 1];
        std::function<void()> after;
        if (chain_launch && active_runs(X_.device) <= 1) {
            const BatchBufs *prev = &X_.bb[slot];
            const bool cut = at2 >= lo_start;
            after = [this, g2, bound, cut, prev] {
                MP_HIP(hipSetDevice(X_.device));
                launch_batch(*g2, bound, cut, prev);
            };
        }
        *ch = Sampler::Chain{g2, B2, slot ^ 1, slot_for(slot ^ 1, B2), std::move(after)};
        *ch_at = at2;
        *ch_B = B2;
        return true;
    };
    bool chain_launched = false; // (the chained batch is on the GPU already)
    while (it < max_total && !done) {
        if (it == lo_start && best_min_score < kMax) {
            ++S->number_lo_iterations;
            // post-LO speculation as after the LOs of the walk below: the batch from
            // lo_starting_iterations on is drawn from the predicted end of the selection
            // stream and launched while the LO steps run (no continuation is pending:
            // batches stop at lo_start)
            bool spec0 = false;
            uint64_t spec0_draws = 0;
            const IterationStream rs_at_lo = rs_;
            const int slot = cur ^ 1;
            const double bound = best_min_score;
            Batch *const gs = &gen[slot];
            const uint32_t at = it;
            bool spec0_chain = false, spec0_chain_launched = false;
            uint32_t spec0_chain_at = 0, spec0_chain_B = 0;
            auto predicted = [this, rs_at_lo, slot, bound, gs, at, max_total, speculate, lo_start, &grow, &batch_size,
                              &spec0, &spec0_draws, &make_chain, &spec0_chain, &spec0_chain_at, &spec0_chain_B,
                              &spec0_chain_launched](const Mt19937 &sel_end) {
                if (!speculate || at >= max_total) return;
                IterationStream from = rs_at_lo;
                from.sel = sel_end;
                slot_free(slot);
                const uint32_t Bs = batch_size(at, sync_batch(grow(at)));
                Sampler::Chain ch;
                spec0_chain = make_chain(at, Bs, slot, bound, &ch, &spec0_chain_at, &spec0_chain_B);
                spec0_chain_launched = spec0_chain && ch.after != nullptr;
                X_.sampler->start(from, gs, Bs, slot, slot_for(slot, Bs),
                                  [this, gs, bound, at, lo_start] {
                                      MP_HIP(hipSetDevice(X_.device));
                                      launch_batch(*gs, bound, at >= lo_start);
                                  },
                                  spec0_chain ? &ch : nullptr);
                spec0 = true;
                spec0_draws = sel_end.draws();
            };
            tl_.mark("lo", (long)it);
            local_opt(S->best_solver_type, best, &S->best_model_score, &S->best_solver_type, predicted);
            tl_.mark("lo_end", spec0 ? 1 : 0);
            termination(*best, max_per);
            if (spec0) {
                if (rs_.sel.draws() == spec0_draws) {
                    tl_.mark("join_spec");
                    have_next = X_.sampler->finish(&rs_);
                    if (have_next) {
                        cur ^= 1;
                        launched = true;
                        // (the chained batch may still be drawing: chained() below)
                        chain_ready = spec0_chain;
                        chain_at = spec0_chain_at;
                        chain_B = spec0_chain_B;
                        chain_launched = spec0_chain && spec0_chain_launched;
                    }
                } else {
                    X_.sampler->cancel();
                    drain_batches(); // a launched speculation drains
                }
            }
        }
        // (drawn here only at the start and after LO / a cut batch: kept short so the
        // GPU starts early and the worker draws the big ones)
        if (!have_next) {
            auto t0 = Clock::now();
            tl_.mark("draw");
            slot_free(cur);
            generate(gen[cur], batch_size(it, sync_batch((uint32_t)bcur)), cur);
            if (gen[cur].B >= 256) draw_s_per_it_ = 0.5 * draw_s_per_it_ + 0.5 * secs(t0) / gen[cur].B;
        }
        auto t_batch = Clock::now();
        const Batch &g = gen[cur];
        const uint32_t B = g.B;
        if (!launched) {
            auto tl = Clock::now();
            tl_.mark("launch", (long)g.B);
            launch_batch(g, best_min_score, it >= lo_start);
            tl_.mark("launched");
            launch_s_ += secs(tl);
            ++launch_n_;
        } else {
            tl_.mark("prelaunched", (long)g.B);
        }
        launched = false;
        BatchBufs &Q = X_.bb[g.slot];
        const bool prof = batch_prof_[g.slot];
        // While the batch is in flight, the sampler thread draws the next one into the
        // other slot.  It is kept if this batch neither triggers LO nor terminates (both
        // rewind the streams); never across lo_start, where an LO runs before the next
        // batch.  Early continuation: the sampler launches it as soon as it is drawn,
        // behind this batch on the stream, instead of after the host has read this one
        // -- the GPU goes straight on.  A batch at or past lo_start that holds a new best
        // runs LO and discards the continuation, and a new best that the device could
        // prove (a published record) makes the continuation's kernels leave at once
        // (the gate), so a discarded continuation costs almost nothing; its bound is this
        // batch's pre-batch best, which is its own unless this batch holds a new best,
        // and then (before lo_start) the bound is conservative and no record skip runs.
        const uint32_t it_next = it + B;
        const uint32_t Bn0 = (it_next < max_total && it_next != lo_start)
                                 ? batch_size(it_next, grow(it_next))
                                 : 0;
        // the chained batch, when it starts where the next one does
        const bool use_chain = chain_ready && Bn0 > 0 && it_next == chain_at;
        if (chain_ready && !use_chain) X_.sampler->cancel(); // (not the next batch)
        chain_ready = false;
        const uint32_t Bn = use_chain ? chain_B : Bn0;
        const bool early = !use_chain && Bn > 0 && early_now(Bn);
        if (Bn > 0 && !use_chain) {
            slot_free(cur ^ 1);
            if (early) {
                Batch *gn = &gen[cur ^ 1];
                const double bound = best_min_score;
                const bool cut_next = it_next >= lo_start;
                const BatchBufs *prev = it >= lo_start ? &Q : nullptr; // this batch can publish a record
                X_.sampler->start(rs_, gn, Bn, cur ^ 1, slot_for(cur ^ 1, Bn), [this, gn, bound, cut_next, prev] {
                    MP_HIP(hipSetDevice(X_.device));
                    launch_batch(*gn, bound, cut_next, prev);
                });
            } else {
                X_.sampler->start(rs_, &gen[cur ^ 1], Bn, cur ^ 1, slot_for(cur ^ 1, Bn));
            }
        }
        auto tw = Clock::now();
        tl_.mark("wait", (long)it);
        MP_HIP(hipEventSynchronize(Q.ev_done));
        tl_.mark("ready");
        S->seconds_gpu_wait += secs(tw);
        batch_s_ = 0.5 * batch_s_ + 0.5 * secs(t_batch);
        S->num_batches++;
        if (prof) {
            float ms_solve = 0.f, ms_score = 0.f;
            MP_HIP(hipEventElapsedTime(&ms_solve, Q.ev[0], Q.ev[1]));
            MP_HIP(hipEventElapsedTime(&ms_score, Q.ev[1], Q.ev[2]));
            tl_.mark("solve_us", (long)(1000.f * ms_solve));
            tl_.mark("score_us", (long)(1000.f * ms_score));
            uint64_t h = 0, trips = 0, scored = 0;
            for (uint32_t q = 0; q < B; ++q) {
                // (record-skipped iterations report their partial trips negated)
                const int c = Q.h_flags8[q] & 0x7f;
                h += (uint64_t)c;
                trips += (uint64_t)std::abs(Q.h_work[q]);
                if (Q.h_work[q] > 0) scored += (uint64_t)c;
            }
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.model_trips += trips;
            g_prof.model_trips_full += h * (uint64_t)((n_ + 255) / 256);
            g_prof.batches += 1;
            g_prof.iterations += B;
            g_prof.hypotheses += h;
            g_prof.scored += scored;
            g_prof.correspondences += h * (uint64_t)n_;
            g_prof.solve_ms += ms_solve;
            g_prof.score_ms += ms_score;
        }

        std::vector<Model> dumped;
        if (model_dump_) {
            dumped.resize((size_t)B * maxm_);
            MP_HIP(hipMemcpyAsync(dumped.data(), Q.d_models, sizeof(Model) * dumped.size(), hipMemcpyDeviceToHost,
                                  X_.copy_stream));
            MP_HIP(hipStreamSynchronize(X_.copy_stream));
        }
        bool invalidated = false;
        bool spec = false; // the sampler holds the post-LO speculation, not the Bn batch
        uint64_t spec_draws = 0;
        bool spec_chain = false, spec_chain_launched = false; // ... and the batch after it (make_chain)
        uint32_t spec_chain_at = 0, spec_chain_B = 0;
        uint32_t j = 0;
        const bool dumping = model_dump_ || count_dump_;
        for (; j < B; ++j) {
            // 64 iterations at a time while nothing happens in them: none marked, not
            // lo_starting_iterations, no solver type reaching its cap (the counts only
            // grow, so a cap reached inside the block is reached at its end)
            while (!dumping && j + 64 <= B && !(lo_start >= it + j && lo_start < it + j + 64)) {
                const uint8_t *f = Q.h_flags8 + j, *ty = g.types.data() + j;
                unsigned mk = 0, n1 = 0, hy = 0;
                for (int k = 0; k < 64; ++k) {
                    mk |= f[k];
                    n1 += ty[k];
                    hy += f[k] & 0x7fu;
                }
                const uint32_t n0 = 64 - n1;
                if ((mk & 0x80u) || S->num_iterations_per_solver[0] + n0 >= max_per[0] ||
                    S->num_iterations_per_solver[1] + n1 >= max_per[1])
                    break;
                S->num_iterations_per_solver[0] += n0;
                S->num_iterations_per_solver[1] += n1;
                S->num_hypotheses += hy;
                j += 64;
            }
            if (j >= B) break;
            const uint32_t iter = it + j;
            const int st = g.types[j];
            S->num_iterations_per_solver[st] += 1;
            const int nm = Q.h_flags8[j] & 0x7f;
            S->num_hypotheses += (uint64_t)nm;
            if (model_dump_) {
                const int32_t hdr[2] = {(int32_t)iter, (int32_t)nm};
                std::fwrite(hdr, sizeof(hdr), 1, model_dump_);
                std::fwrite(dumped.data() + (size_t)j * maxm_, sizeof(Model), (size_t)nm, model_dump_);
            }
            if (count_dump_) {
                const int *smp = slot_ptr(g.slot) + 8 * (size_t)j;
                std::fprintf(count_dump_, "%u %d %d", iter, st, nm);
                for (int q = 0; q < (st == 0 ? ss_[0][0] : ss_[1][2]); ++q) std::fprintf(count_dump_, " %d", smp[q]);
                std::fprintf(count_dump_, "\n");
            }
            bool lo_here = false;
            if (nm > 0) {
                // The device sums screen; the decision is taken on reference-order sums
                // (exact_score) -- see resolve_tie.  `maybe`: the iteration could hold a new
                // best (some model's lower bound is below the running best, or no bound
                // holds); `certain`: it does, and its best model is the reference's winner.
                // Unmarked iterations (flag byte without 0x80) cannot: their lo is at or
                // above the pre-batch best, which bounds the running best from above.
                const bool marked = (Q.h_flags8[j] & 0x80) != 0;
                const IterResult &res = Q.h_cand[j]; // (valid when marked)
                const double bl = marked ? res.best : kMax;
                const int raw = marked ? res.slot : 0;
                const bool uncertain = (raw & kSlotUncertain) != 0;
                const bool maybe = marked && (uncertain || (best_min_score == kMax ? bl < kMax : res.lo < best_min_score));
                if (maybe || iter == lo_start) {
                    bool new_best = false;
                    if (maybe) {
                        const bool certain = !uncertain && !(raw & kSlotAmbiguous) &&
                                             (best_min_score == kMax || res.hi < best_min_score);
                        Model m;
                        double e = kMax;
                        if (certain) {
                            m = fetch_model(Q, (int)j);
                            tl_.mark("exact", (long)iter);
                            e = exact_score(m);  // (below best_min_score: the bounds say so)
                        } else {
                            tl_.mark("resolve", (long)iter);
                            resolve_tie(Q, j, &m, &e);
                        }
                        tl_.mark("decided", e < best_min_score ? 1 : 0);
                        if (e < best_min_score) {
                            new_best = true;
                            best_min = m;
                            best_min_score = e;
                        }
                    }
                    if (new_best) {
                        if (trace_) std::fprintf(stderr, "[engine] it=%u new best %.17g (device %.17g, solver %d, %d models)\n",
                                                 iter, best_min_score, bl, st, nm);
                        update_best(best_min_score, best_min, st, &S->best_model_score, best, &S->best_solver_type);
                    }
                    // the reference enters this block only on a new best or at
                    // lo_starting_iterations (src/hybrid_ransac.h:123-124); a `maybe` that
                    // the exact sums reject is no entry
                    const bool run_lo = (new_best || iter == lo_start) && iter >= lo_start && best_min_score < kMax;
                    if (new_best || run_lo) {
                        if (run_lo) {
                            // rewind both streams to the end of iteration `iter`
                            rewind(g, j);
                            ++S->number_lo_iterations;
                            double sc = best_min_score;
                            const uint32_t at = iter + 1;
                            // The hook runs on an LO worker beside the steps: it
                            // gets copies of the loop state it reads -- the streams as rewound
                            // (the LO draws only from its own copies of the selection stream
                            // and writes rs_ after LoWorkers::run has returned), the free
                            // slot, whether a continuation is pending, the pre-LO best (LO
                            // leaves best_min_model_score alone, src/hybrid_ransac.h:149-155)
                            // -- and writes only spec / spec_draws, read after the join.
                            const IterationStream rs_at_lo = rs_;
                            const int slot = cur ^ 1;
                            const bool cont_pending = Bn > 0;
                            const double bound = best_min_score;
                            Batch *const gs = &gen[slot];
                            auto predicted = [this, rs_at_lo, slot, cont_pending, bound, gs, at, max_total, speculate,
                                              lo_start, &grow, &batch_size, &spec, &spec_draws, &make_chain,
                                              &spec_chain, &spec_chain_at, &spec_chain_B,
                                              &spec_chain_launched](const Mt19937 &sel_end) {
                                if (!speculate || at >= max_total) return;
                                if (cont_pending) X_.sampler->cancel(); // the no-LO continuation
                                IterationStream from = rs_at_lo;
                                from.sel = sel_end;
                                const uint32_t bc = grow(at);
                                slot_free(slot); // (an early continuation's samples are on the device)
                                const uint32_t Bs = batch_size(at, sync_batch(bc));
                                Sampler::Chain ch;
                                spec_chain = make_chain(at, Bs, slot, bound, &ch, &spec_chain_at, &spec_chain_B);
                                spec_chain_launched = spec_chain && ch.after != nullptr;
                                X_.sampler->start(from, gs, Bs, slot, slot_for(slot, Bs),
                                                  [this, gs, bound, at, lo_start] {
                                                      // the sampler thread is not bound to the
                                                      // estimator's device by itself
                                                      MP_HIP(hipSetDevice(X_.device));
                                                      launch_batch(*gs, bound, at >= lo_start);
                                                  },
                                                  spec_chain ? &ch : nullptr);
                                spec = true;
                                spec_draws = sel_end.draws();
                            };
                            tl_.mark("lo", (long)iter);
                            local_opt(S->best_solver_type, &best_min, &sc, &S->best_solver_type, predicted);
                            tl_.mark("lo_end", spec ? 1 : 0);
                            if (trace_) std::fprintf(stderr, "[engine] it=%u LO %.17g -> %.17g\n", iter, best_min_score, sc);
                            update_best(sc, best_min, st, &S->best_model_score, best, &S->best_solver_type);
                            lo_here = true;
                            invalidated = true;
                        }
                        termination(*best, max_per);
                    }
                }
            }
            if (S->num_iterations_per_solver[st] >= max_per[st]) {
                // `break` in the reference skips the loop increment
                S->num_iterations_total = iter;
                done = true;
                if (!lo_here) rewind(g, j);
                break;
            }
            if (invalidated) {
                it = iter + 1;
                break;
            }
        }
        if (!done && !invalidated) {
            it += B;
            have_next = false;
            if (Bn > 0 && use_chain) { // drawn during the LO and the walk (chained speculation)
                tl_.mark("chained", (long)Bn);
                IterationStream crs;
                if (X_.sampler->chained(&crs)) {
                    tl_.mark("chain_joined");
                    rs_ = crs;
                    have_next = true;
                    cur ^= 1;
                    launched = chain_launched;
                } // (else rs_ stands at the end of this batch)
            } else if (Bn > 0) { // rs_ moves to the end of the drawn batch
                auto t0 = Clock::now();
                tl_.mark("join_sampler");
                have_next = X_.sampler->finish(&rs_);
                tl_.mark("joined", have_next ? 1 : 0);
                sample_s_ += secs(t0);
                if (have_next) {
                    cur ^= 1;
                    launched = early; // (the sampler launched it once drawn)
                }
            }
            // (otherwise rs_ stands at the end of this batch)
        } else if (spec) {
            have_next = false;
            if (!done && rs_.sel.draws() == spec_draws) {
                // the LO ended where predicted: the speculative batch comes next
                tl_.mark("join_spec");
                have_next = X_.sampler->finish(&rs_);
                tl_.mark("joined", have_next ? 1 : 0);
                if (have_next) {
                    cur ^= 1;
                    launched = true;
                    chain_ready = spec_chain; // (still drawing, maybe: chained() above)
                    chain_at = spec_chain_at;
                    chain_B = spec_chain_B;
                    chain_launched = spec_chain && spec_chain_launched;
                }
            } else {
                X_.sampler->cancel();
                drain_batches(); // a launched speculation drains
            }
        } else {
            if (Bn > 0) X_.sampler->cancel();
            have_next = false;
        }
        bcur = (int)grow(it);
    }
    if (!done) S->num_iterations_total = it;
    // (a continuation launched past the end may still be in flight: the next run reuses
    // the buffers)
    X_.sampler->cancel();
    drain_batches();

    if (S->num_iterations_total <= lo_start && S->best_model_score < kMax) {
        ++S->number_lo_iterations;
        local_opt(S->best_solver_type, best, &S->best_model_score, &S->best_solver_type);
        termination(*best, max_per);
    }
    if (o_.final_least_squares) {
        auto t0 = Clock::now();
        Model refined = *best;
        least_squares(lanes_[0], S->inlier_indices, &refined, false);
        double sc;
        if (score_below(lanes_[0], refined, S->best_model_score, &sc) && sc < S->best_model_score) {
            S->best_model_score = sc;
            *best = refined;
            termination(*best, max_per);
        }
        S->seconds_lo += secs(t0);
    }
    S->seconds_total = secs(t_start);
    tl_.mark("end");
    for (const auto &e : tl_.ev) std::fprintf(stderr, "[timeline %ld] %10.1f %-14s %ld\n", tl_.run, e.us, e.what, e.a);
    double tsum[3] = {0, 0, 0};
    for (const Lane &L : lanes_) {
        S->num_lo_sweeps += L.count;
        for (int k = 0; k < 3; ++k) tsum[k] += L.t[k];
    }
    if (std::getenv("MADPOSE_LO_TIMING"))
        std::fprintf(stderr, "[engine] pair: %.1f us total, %d batches (%d launched by the estimator thread, %.1f us "
                     "each), gpu wait %.1f us, sampling %.1f us, LO %.1f us\n", 1e6 * S->seconds_total,
                     (int)S->num_batches, launch_n_, launch_n_ ? 1e6 * launch_s_ / launch_n_ : 0.0,
                     1e6 * S->seconds_gpu_wait, 1e6 * sample_s_, 1e6 * S->seconds_lo);
    if (std::getenv("MADPOSE_LO_TIMING") && lo_t_[2] > 0)
        std::fprintf(stderr, "[engine] %d LO: prefix %.1f us, steps %.1f us, step sum %.1f us, step0 %.1f us, longest "
                     "step %.1f us, step0 fit %.1f us, step0 score %.1f us, other fit %.1f us, step0 lsq %.1f us, "
                     "step0 iters %.1f us, other lsq %.1f us, other iters %.1f us (avg per LO), recomputed %.2f us\n",
                     (int)lo_t_[2], 1e6 * lo_t_[0] / lo_t_[2], 1e6 * lo_t_[1] / lo_t_[2], 1e6 * lo_t_[3] / lo_t_[2],
                     1e6 * lo_t_[5] / lo_t_[2], 1e6 * lo_t_[4], 1e6 * lo_t_[6] / lo_t_[2], 1e6 * lo_t_[7] / lo_t_[2],
                     1e6 * lo_t_[8] / lo_t_[2], 1e6 * lo_t_[9] / lo_t_[2], 1e6 * lo_t_[10] / lo_t_[2],
                     1e6 * lo_t_[11] / lo_t_[2], 1e6 * lo_t_[12] / lo_t_[2], lo_t_[13] / lo_t_[2]);
    if (lo_timing_ && lm_stat_[0] > 0)
        std::fprintf(stderr, "[engine] %d big LM solves: %.1f evaluations, %.0f blocks, %.1f us each (avg)\n",
                     (int)lm_stat_[0], lm_stat_[1] / lm_stat_[0], lm_stat_[3] / lm_stat_[0], 1e6 * lm_stat_[2] / lm_stat_[0]);
    if (std::getenv("MADPOSE_LO_TIMING") && lo_t_[2] > 0)
        std::fprintf(stderr, "[engine] LO steps phase: before the parallel run %.1f us, the run %.1f us, the speculation "
                     "hook %.1f us (avg per LO)\n",
                     1e6 * lo_seg_[0] / lo_t_[2], 1e6 * lo_seg_[1] / lo_t_[2], 1e6 * lo_seg_[2] / lo_t_[2]);
    if (std::getenv("MADPOSE_SWEEP_TIMING") && S->num_lo_sweeps > 0)
        std::fprintf(stderr, "[engine] %llu host sweeps: %.2f us (avg)\n", (unsigned long long)S->num_lo_sweeps,
                     1e6 * tsum[1] / S->num_lo_sweeps);
    if (g_prof_on.load(std::memory_order_relaxed)) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof.sample_wall_ms += 1e3 * sample_s_;
        g_prof.wait_wall_ms += 1e3 * S->seconds_gpu_wait;
        g_prof.run_wall_ms += 1e3 * S->seconds_total;
        g_prof.accepted += S->num_hypotheses;
        g_prof.tie_checks += tie_checks_;
    }
}

void validate(const PairInput &in, const RansacOptions &o) {
    if (in.variant < 0 || in.variant > 3)
        throw std::invalid_argument("variant must be 0 (calibrated), 1 (shared focal), 2 (two focal) or 3 (scale only)");
    if (in.n < 0 || in.n > (int64_t)1 << 30) throw std::invalid_argument("bad number of correspondences");
    if (in.n > 0 && (!in.x0 || !in.x1 || !in.d0 || !in.d1)) throw std::invalid_argument("null input array");
    if (!(o.squared_inlier_thresholds[0] > 0) || !(o.squared_inlier_thresholds[1] > 0))
        throw std::invalid_argument("squared_inlier_thresholds must hold two positive values");

}

} // namespace

// (MADPOSE_PROF_OFF=1: profiling stays off whatever the caller asks -- A/B of its cost)
void profile_enable(bool on) {
    static const bool off = [] {
        return env_flag("MADPOSE_PROF_OFF", false);
    }();
    g_prof_on.store(on && !off);
}
void profile_reset() {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof = KernelProfile();
}
KernelProfile profile_read() {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    return g_prof;
}

void estimate_pair(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int device, Model *out,
                   Stats *stats) {
    validate(in, opts);
    CtxLease lease(device);
    Problem P = make_problem(in, opts, cfg);
    Run r(*lease.c, P, opts, cfg);
    r.run(out, stats);
    if (in.variant == kSF) {
        out->focal0 *= P.norm_scale;
        out->focal1 = out->focal0;
    } else if (in.variant == kTF) {
        out->focal0 *= P.norm_scale;
        out->focal1 *= P.norm_scale;
    }
}

namespace {
// device allocation freed on scope exit (error paths included)
template <class T> struct DevArray {
    T *p = nullptr;
    explicit DevArray(size_t n) { MP_HIP(hipMalloc(&p, sizeof(T) * std::max<size_t>(n, 1))); }
    ~DevArray() {
        if (p) hipFree(p);
    }
    DevArray(const DevArray &) = delete;
    DevArray &operator=(const DevArray &) = delete;
};
} // namespace

void score_models(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                  int nm, double *scores, double *errors, int device, double *norm_scale) {
    validate(in, opts);
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    Problem P = make_problem(in, opts, cfg);
    if (norm_scale) *norm_scale = P.norm_scale;
    X.ensure(in.n, 64, max_models(in.variant == kScaleOnly ? kCal : in.variant));
    PairData D;
    upload_pair(X, P, &D);
    std::vector<ScoreRec> recs(std::max(nm, 1));
    for (int m = 0; m < nm; ++m) prepare_score_rec(P.C, models[m], recs[m]);
    DevArray<ScoreRec> d_recs(recs.size());
    DevArray<double> d_sc(recs.size());
    MP_HIP(hipMemcpyAsync(d_recs.p, recs.data(), sizeof(ScoreRec) * nm, hipMemcpyHostToDevice, X.stream));
    MP_HIP(launch_score_models(X.stream, D, P.C, d_recs.p, nm, d_sc.p));
    MP_HIP(hipMemcpyAsync(scores, d_sc.p, sizeof(double) * nm, hipMemcpyDeviceToHost, X.stream));
    if (errors) {
        for (int m = 0; m < nm; ++m) {
            MP_HIP(launch_sweep(X.stream, D, P.C, d_recs.p + m, X.d_err, X.d_score1));
            MP_HIP(hipMemcpyAsync(errors + (size_t)m * 3 * in.n, X.d_err, sizeof(double) * 3 * in.n,
                                  hipMemcpyDeviceToHost, X.stream));
        }
    }
    MP_HIP(hipStreamSynchronize(X.stream));
}

// score_batch's per-correspondence errors and flags of explicit models, with each
// model's per-term bounds and margin (mp_debug_score_terms; test hook of the screening
// margins, mp_score.h score_margins)
void debug_score_terms(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                       int nm, double *errors, int *flags, double *taus, double *ties, int device) {
    validate(in, opts);
    if (nm <= 0) return;
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    Problem P = make_problem(in, opts, cfg);
    X.ensure(in.n, 64, max_models(in.variant == kScaleOnly ? kCal : in.variant));
    PairData D;
    upload_pair(X, P, &D);
    std::vector<ScoreRec> recs(nm);
    for (int m = 0; m < nm; ++m) {
        prepare_score_rec(P.C, models[m], recs[m], taus ? taus + 3 * m : nullptr);
        if (ties) ties[m] = recs[m].tie;
    }
    DevArray<ScoreRec> d_recs(nm);
    DevArray<double> d_err((size_t)nm * 3 * in.n);
    DevArray<int> d_flags((size_t)nm * in.n);
    MP_HIP(hipMemcpyAsync(d_recs.p, recs.data(), sizeof(ScoreRec) * nm, hipMemcpyHostToDevice, X.stream));
    MP_HIP(launch_debug_terms(X.stream, D, P.C, d_recs.p, nm, d_err.p, d_flags.p));
    MP_HIP(hipMemcpyAsync(errors, d_err.p, sizeof(double) * nm * 3 * in.n, hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(flags, d_flags.p, sizeof(int) * nm * in.n, hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
}

void lo_sweep_models(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                     int nm, double *scores, double *errors, double *fast_bounds) {
    validate(in, opts);
    Problem P = make_problem(in, opts, cfg);
    LoSweepData D;
    lo_sweep_prepare(P.C, P.H.x0.data(), P.H.x1.data(), P.H.d0.data(), P.H.d1.data(), &D);
    std::vector<double> err(3 * (size_t)std::max<int64_t>(in.n, 1));
    for (int m = 0; m < nm; ++m) {
        scores[m] = lo_sweep(P.C, D, models[m], err.data());
        if (errors) std::memcpy(errors + (size_t)m * 3 * in.n, err.data(), sizeof(double) * 3 * in.n);
        if (fast_bounds) lo_sweep_fast(P.C, D, models[m], err.data(), fast_bounds + 2 * m, fast_bounds + 2 * m + 1);
    }
}

// score_batch on explicit per-iteration model lists (mp_debug_score_batch, test hook):
// the estimator's launch with the pre-batch best `best`, and the exact early exit /
// record skip as flags allow; results, bounds, margins and record models back
void debug_score_batch(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nb,
                       const int *counts, const Model *models, double best, int flags, double *res_best,
                       int *res_slot, Model *rec_models, double *res_hi_lo, double *model_ties, int device) {
    validate(in, opts);
    const int v = in.variant == kScaleOnly ? kCal : in.variant;
    const int maxm = max_models(v);
    if (nb <= 0 || nb > (1 << 20)) throw std::invalid_argument("bad iteration count");
    for (int b = 0; b < nb; ++b)
        if (counts[b] < 0 || counts[b] > maxm) throw std::invalid_argument("model count out of range");
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    Problem P = make_problem(in, opts, cfg);
    X.ensure(in.n, nb, maxm);
    PairData D;
    upload_pair(X, P, &D);
    BatchBufs &Q = X.bb[0];
    std::vector<ScoreRec> recs((size_t)nb * maxm);
    std::vector<Model> ms((size_t)nb * maxm);
    std::memset(ms.data(), 0, sizeof(Model) * ms.size());
    std::memset(recs.data(), 0, sizeof(ScoreRec) * recs.size());
    for (int b = 0; b < nb; ++b)
        for (int m = 0; m < counts[b]; ++m) {
            ms[(size_t)b * maxm + m] = models[(size_t)b * maxm + m];
            prepare_score_rec(P.C, ms[(size_t)b * maxm + m], recs[(size_t)b * maxm + m]);
        }
    if (model_ties)
        for (size_t k = 0; k < recs.size(); ++k) model_ties[k] = recs[k].tie;
    MP_HIP(hipMemcpyAsync(Q.d_recs, recs.data(), sizeof(ScoreRec) * recs.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(hipMemcpyAsync(Q.d_models, ms.data(), sizeof(Model) * ms.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(hipMemcpyAsync(Q.d_counts, counts, sizeof(int) * nb, hipMemcpyHostToDevice, X.stream));
    std::memset(Q.h_recmodel, 0, sizeof(Model) * nb);
    const bool exit = (flags & 1) != 0, skip = (flags & 2) != 0;
    const unsigned epoch_hi = ~(++X.epoch);
    MP_HIP(launch_score_batch(X.stream, D, P.C, Q.d_recs, Q.d_counts, nb, maxm, Q.d_scores, Q.d_res,
                              exit ? best : DBL_MAX, nullptr, skip ? X.d_recword : nullptr, epoch_hi, Q.d_models,
                              Q.d_recmodel));
    std::vector<IterResult> res(nb);
    MP_HIP(hipMemcpyAsync(res.data(), Q.d_res, sizeof(IterResult) * nb, hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
    for (int b = 0; b < nb; ++b) {
        res_best[b] = res[b].best;
        res_slot[b] = res[b].slot;
        if (res_hi_lo) {
            res_hi_lo[2 * b] = res[b].hi;
            res_hi_lo[2 * b + 1] = res[b].lo;
        }
    }
    if (rec_models) std::memcpy(rec_models, Q.h_recmodel, sizeof(Model) * nb);
}

namespace {
// the problem lists of mp_lm_refine_batch: offsets[0] >= 0, non-decreasing, every
// index inside the pair (checked once, before either LM touches them)
void validate_lm_batch(const PairInput &in, int nprob, const int64_t *offsets, const int32_t *idx, const Model *models,
                       const int32_t *status) {
    if (nprob < 0) throw std::invalid_argument("negative problem count");
    if (nprob == 0) return;
    if (!offsets || !models || !status) throw std::invalid_argument("null offsets, models or status");
    if (offsets[0] < 0) throw std::invalid_argument("sample offsets must be non-negative");
    for (int64_t k = 0; k < 3 * (int64_t)nprob; ++k)
        if (offsets[k + 1] < offsets[k]) throw std::invalid_argument("sample offsets must not decrease");
    if (offsets[3 * (int64_t)nprob] > offsets[0] && !idx) throw std::invalid_argument("null index list");
    for (int64_t k = offsets[0]; k < offsets[3 * (int64_t)nprob]; ++k)
        if (idx[k] < 0 || idx[k] >= in.n) throw std::invalid_argument("sample index out of range");
}
} // namespace

// the same problems through the host LM (host/lm.cpp) -- test hook (mp_debug_lm_refine_host);
// kinds may be NULL (every problem a LeastSquares call)
void lm_refine_batch_host(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nprob,
                          const int32_t *kinds, const int64_t *offsets, const int32_t *idx, Model *models,
                          int32_t *status) {
    validate(in, opts);
    validate_lm_batch(in, nprob, offsets, idx, models, status);
    Problem P = make_problem(in, opts, cfg);
    const int v = P.C.variant;
    const int kmd = v == kCal ? 3 : 4, kpt = v == kCal ? 5 : (v == kSF ? 6 : 7);
    for (int j = 0; j < nprob; ++j) {
        std::vector<int> smp[3];
        int sz[3];
        for (int t = 0; t < 3; ++t) {
            smp[t].assign(idx + offsets[3 * j + t], idx + offsets[3 * j + t + 1]);
            sz[t] = (int)smp[t].size();
        }
        if ((sz[0] < kmd && sz[1] < kmd) || sz[2] < kpt) {
            status[j] = 3;
            continue;
        }
        const LmJob J = make_lm_job(P, cfg, sz, 0, kinds && kinds[j] == 1, models[j]);
        LMSettings S;
        S.use_reproj = cfg.lo_type != 1;
        S.use_sampson = cfg.lo_type != 2;
        S.use_shift = J.use_shift != 0;
        S.min_depth_constraint = J.min_depth_constraint != 0;
        S.w_sampson = J.w_sampson;
        S.ftol = J.ftol;
        S.gtol = J.gtol;
        S.ptol = J.ptol;
        S.max_iter = J.max_iter;
        S.nonmonotonic = J.nonmonotonic != 0;
        status[j] = lm_refine(P.H, smp, S, &models[j]) ? 1 : 0;
    }
}

void lm_refine_batch_device(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nprob,
                            const int32_t *kinds, const int64_t *offsets, const int32_t *idx, Model *models,
                            int32_t *status, int device) {
    validate(in, opts);
    validate_lm_batch(in, nprob, offsets, idx, models, status);
    if (nprob <= 0) return;
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    Problem P = make_problem(in, opts, cfg);
    X.ensure(in.n, 64, max_models(in.variant == kScaleOnly ? kCal : in.variant));
    PairData D;
    upload_pair(X, P, &D);
    const int v = P.C.variant;
    const int kmd = v == kCal ? 3 : 4, kpt = v == kCal ? 5 : (v == kSF ? 6 : 7);
    std::vector<LmJob> jobs;
    std::vector<int> which;
    for (int j = 0; j < nprob; ++j) {
        int sz[3];
        for (int t = 0; t < 3; ++t) sz[t] = (int)(offsets[3 * j + t + 1] - offsets[3 * j + t]);
        // too few data for the solver (the size test of least_squares)
        if ((sz[0] < kmd && sz[1] < kmd) || sz[2] < kpt) {
            status[j] = 3;
            continue;
        }
        jobs.push_back(make_lm_job(P, cfg, sz, (int)offsets[3 * j], kinds && kinds[j] == 1, models[j]));
        which.push_back(j);
    }
    if (jobs.empty()) return;
    const int64_t nidx = offsets[3 * nprob];
    DevArray<LmJob> d_jobs(jobs.size());
    DevArray<int> d_idx((size_t)nidx), d_status(jobs.size());
    DevArray<Model> d_out(jobs.size());
    MP_HIP(hipMemcpyAsync(d_jobs.p, jobs.data(), sizeof(LmJob) * jobs.size(), hipMemcpyHostToDevice, X.stream));
    if (nidx > 0) MP_HIP(hipMemcpyAsync(d_idx.p, idx, sizeof(int) * nidx, hipMemcpyHostToDevice, X.stream));
    MP_HIP(launch_lm_batch(X.stream, D, P.C, d_jobs.p, (int)jobs.size(), d_idx.p, d_out.p, d_status.p));
    std::vector<Model> out(jobs.size());
    std::vector<int> st(jobs.size());
    MP_HIP(hipMemcpyAsync(out.data(), d_out.p, sizeof(Model) * out.size(), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(st.data(), d_status.p, sizeof(int) * st.size(), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
    for (size_t k = 0; k < which.size(); ++k) {
        models[which[k]] = out[k];
        status[which[k]] = st[k];
    }
}

int solve_md_direct(int variant, const double *x, const double *y, const double *dx, const double *dy, double *sols,
                    int max_sols, Model *poses, int max_poses, int *nposes, int device, int alt) {
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    const int k = variant == kCal ? 3 : 4;
    std::vector<double> in(8 * k);
    std::memcpy(in.data(), x, sizeof(double) * 3 * k);
    std::memcpy(in.data() + 3 * k, y, sizeof(double) * 3 * k);
    std::memcpy(in.data() + 6 * k, dx, sizeof(double) * k);
    std::memcpy(in.data() + 7 * k, dy, sizeof(double) * k);
    DevArray<double> d_in(in.size()), d_sols(8 * 6);
    DevArray<int> d_n(2);
    DevArray<Model> d_poses(8);
    MP_HIP(hipMemcpyAsync(d_in.p, in.data(), sizeof(double) * in.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(launch_md_direct(X.stream, variant, alt, d_in.p, d_sols.p, d_n.p, d_poses.p, d_n.p + 1));
    double hs[48];
    int hn[2];
    Model hp[8];
    MP_HIP(hipMemcpyAsync(hs, d_sols.p, sizeof(hs), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(hn, d_n.p, sizeof(hn), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(hp, d_poses.p, sizeof(hp), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
    const int w = variant == kCal ? 4 : (variant == kSF ? 5 : 6);
    for (int i = 0; i < std::min(hn[0], max_sols); ++i)
        for (int c = 0; c < w; ++c) sols[i * w + c] = hs[i * w + c];
    for (int i = 0; i < std::min(hn[1], max_poses); ++i) poses[i] = hp[i];
    if (nposes) *nposes = hn[1];
    return hn[0];
}

int solve_point_direct(int kind, const double *x1, const double *x2, Model *poses, int max_poses, int device) {
    if (kind < 0 || kind > 2) throw std::invalid_argument("point solver kind must be 0, 1 or 2");
    if (kind == 1) {
        // the estimator's root stage (deflated eigenproblem) on this one sample, then
        // its poses
        double cand[kPtCandStride];
        int nc = 0;
        debug_pt_roots(kSF, 1, x1, x2, cand, &nc, device);
        CtxLease lease(device);
        DeviceCtx &X = *lease.c;
        double in[24];
        std::memcpy(in, x1, sizeof(double) * 12);
        std::memcpy(in + 12, x2, sizeof(double) * 12);
        constexpr int kCap = 16;
        DevArray<double> d_in(24), d_cand(kPtCandStride);
        DevArray<int> d_nc(1), d_n(1);
        DevArray<Model> d_poses(kCap);
        MP_HIP(hipMemcpyAsync(d_in.p, in, sizeof(in), hipMemcpyHostToDevice, X.stream));
        MP_HIP(hipMemcpyAsync(d_cand.p, cand, sizeof(cand), hipMemcpyHostToDevice, X.stream));
        MP_HIP(hipMemcpyAsync(d_nc.p, &nc, sizeof(int), hipMemcpyHostToDevice, X.stream));
        MP_HIP(launch_point_direct_6pt(X.stream, d_in.p, d_cand.p, d_nc.p, d_poses.p, d_n.p));
        int hn = 0;
        Model hp[kCap];
        MP_HIP(hipMemcpyAsync(&hn, d_n.p, sizeof(int), hipMemcpyDeviceToHost, X.stream));
        MP_HIP(hipMemcpyAsync(hp, d_poses.p, sizeof(hp), hipMemcpyDeviceToHost, X.stream));
        MP_HIP(hipStreamSynchronize(X.stream));
        for (int i = 0; i < std::min(std::min(hn, kCap), max_poses); ++i) poses[i] = hp[i];
        return hn;
    }
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    const int per = kind == 0 ? 15 : 14;
    double in[30];
    std::memcpy(in, x1, sizeof(double) * per);
    std::memcpy(in + per, x2, sizeof(double) * per);
    constexpr int kCap = 16;
    DevArray<double> d_in(30), d_cand(kPtCandStride);
    DevArray<int> d_n(1), d_nc(1);
    DevArray<Model> d_poses(kCap);
    MP_HIP(hipMemcpyAsync(d_in.p, in, sizeof(in), hipMemcpyHostToDevice, X.stream));
    MP_HIP(launch_point_direct(X.stream, kind, d_in.p, d_poses.p, d_n.p, d_cand.p, d_nc.p));
    int hn = 0;
    Model hp[kCap];
    MP_HIP(hipMemcpyAsync(&hn, d_n.p, sizeof(int), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(hp, d_poses.p, sizeof(hp), hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
    for (int i = 0; i < std::min(std::min(hn, kCap), max_poses); ++i) poses[i] = hp[i];
    return hn;
}

void debug_pt_roots(int variant, int64_t ns, const double *pts0, const double *pts1, double *cand, int *ncand,
                    int device) {
    if (variant != kCal && variant != kSF && variant != kTF)
        throw std::invalid_argument("variant must be 0 (5pt), 1 (6pt) or 2 (7pt)");
    if (ns <= 0 || ns > (1 << 22)) throw std::invalid_argument("bad number of samples");
    CtxLease lease(device);
    DeviceCtx &X = *lease.c;
    const int K = variant == kCal ? 5 : (variant == kSF ? 6 : 7);
    const int64_t np = K * ns;
    // one correspondence per sample point, identity intrinsics, sample s = points Ks..Ks+K-1
    std::vector<double> host(8 * (size_t)np);
    for (int64_t i = 0; i < np; ++i) {
        host[i] = pts0[2 * i];
        host[np + i] = pts0[2 * i + 1];
        host[2 * np + i] = pts1[2 * i];
        host[3 * np + i] = pts1[2 * i + 1];
        host[4 * np + i] = host[5 * np + i] = 1.0;
        host[6 * np + i] = 1.0 / std::sqrt(pts0[2 * i] * pts0[2 * i] + pts0[2 * i + 1] * pts0[2 * i + 1] + 1.0);
        host[7 * np + i] = 1.0 / std::sqrt(pts1[2 * i] * pts1[2 * i] + pts1[2 * i + 1] * pts1[2 * i + 1] + 1.0);
    }
    std::vector<int> smp(8 * (size_t)ns, 0), list(ns);
    for (int64_t s = 0; s < ns; ++s) {
        list[s] = (int)s;
        for (int j = 0; j < K; ++j) smp[8 * s + j] = (int)(K * s + j);
    }
    DevArray<double> d_pair_a(host.size()), d_cand_a(kPtCandStride * (size_t)ns);
    DevArray<int> d_smp_a(smp.size()), d_list_a(list.size()), d_n_a((size_t)ns);
    double *d_pair = d_pair_a.p, *d_cand = d_cand_a.p;
    int *d_smp = d_smp_a.p, *d_list = d_list_a.p, *d_n = d_n_a.p;
    MP_HIP(hipMemcpyAsync(d_pair, host.data(), sizeof(double) * host.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(hipMemcpyAsync(d_smp, smp.data(), sizeof(int) * smp.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(hipMemcpyAsync(d_list, list.data(), sizeof(int) * list.size(), hipMemcpyHostToDevice, X.stream));
    MP_HIP(hipMemsetAsync(d_cand, 0, sizeof(double) * kPtCandStride * (size_t)ns, X.stream));
    PairData D{d_pair, d_pair + np, d_pair + 2 * np, d_pair + 3 * np, d_pair + 4 * np, d_pair + 5 * np,
               d_pair + 6 * np, d_pair + 7 * np};
    PairConst C{};
    C.variant = variant;
    C.n = (int)np;
    for (int k = 0; k < 9; ++k) C.K0[k] = C.K1[k] = C.K0i[k] = C.K1i[k] = (k % 4 == 0) ? 1.0 : 0.0;
    DevArray<double> d_pen(variant == kSF ? (size_t)ns * kPtPenStride : 1);
    MP_HIP(launch_pt_roots(X.stream, D, C, d_list, (int)ns, d_smp, d_cand, d_n, d_pen.p));
    MP_HIP(hipMemcpyAsync(cand, d_cand, sizeof(double) * kPtCandStride * (size_t)ns, hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipMemcpyAsync(ncand, d_n, sizeof(int) * (size_t)ns, hipMemcpyDeviceToHost, X.stream));
    MP_HIP(hipStreamSynchronize(X.stream));
}

void bougnoux_batch(int64_t k, const double *F, double *out, int device) {
    if (k <= 0) return;
    CtxLease lease(device);
    hipStream_t s = lease.c->stream;
    DevArray<double> d_F(9 * (size_t)k), d_out(2 * (size_t)k);
    MP_HIP(hipMemcpyAsync(d_F.p, F, sizeof(double) * 9 * (size_t)k, hipMemcpyHostToDevice, s));
    MP_HIP(launch_bougnoux(s, d_F.p, k, d_out.p));
    MP_HIP(hipMemcpyAsync(out, d_out.p, sizeof(double) * 2 * (size_t)k, hipMemcpyDeviceToHost, s));
    MP_HIP(hipStreamSynchronize(s));
}

void pose_eval_batch(int64_t k, const double *R, const double *t, const double *T, double t_thres, double *err_t,
                     double *err_R, int nthr, const double *thr, double *aucs, int device) {
    if (k <= 0) {
        for (int b = 0; b < nthr; ++b) aucs[b] = NAN;
        return;
    }
    CtxLease lease(device);
    hipStream_t s = lease.c->stream;
    // one block: R (9k) t (3k) T (16k) | err_t err_R max(err_t, err_R) sorted (4k) | thr, aucs (2 nthr)
    const size_t in = 28 * (size_t)k, tot = in + 4 * (size_t)k + 2 * (size_t)std::max(nthr, 0);
    std::vector<double> host(in);
    std::memcpy(host.data(), R, sizeof(double) * 9 * k);
    std::memcpy(host.data() + 9 * k, t, sizeof(double) * 3 * k);
    std::memcpy(host.data() + 12 * k, T, sizeof(double) * 16 * k);
    DevArray<double> d_all(tot);
    double *d = d_all.p;
    double *d_et = d + in, *d_eR = d_et + k, *d_max = d_eR + k, *d_sorted = d_max + k, *d_thr = d_sorted + k,
           *d_auc = d_thr + nthr;
    MP_HIP(hipMemcpyAsync(d, host.data(), sizeof(double) * in, hipMemcpyHostToDevice, s));
    if (nthr > 0) MP_HIP(hipMemcpyAsync(d_thr, thr, sizeof(double) * nthr, hipMemcpyHostToDevice, s));
    MP_HIP(launch_pose_errors(s, k, d, d + 9 * k, d + 12 * k, t_thres, d_et, d_eR, nthr > 0 ? d_max : nullptr));
    MP_HIP(launch_pose_auc(s, k, d_max, d_sorted, nthr, d_thr, d_auc));
    MP_HIP(hipMemcpyAsync(err_t, d_et, sizeof(double) * k, hipMemcpyDeviceToHost, s));
    MP_HIP(hipMemcpyAsync(err_R, d_eR, sizeof(double) * k, hipMemcpyDeviceToHost, s));
    if (nthr > 0) MP_HIP(hipMemcpyAsync(aucs, d_auc, sizeof(double) * nthr, hipMemcpyDeviceToHost, s));
    MP_HIP(hipStreamSynchronize(s));
}

void pose_auc_batch(int64_t k, const double *errors, int nthr, const double *thr, double *aucs, int device) {
    if (nthr <= 0) return;
    if (k <= 0) {
        for (int b = 0; b < nthr; ++b) aucs[b] = NAN;
        return;
    }
    CtxLease lease(device);
    hipStream_t s = lease.c->stream;
    DevArray<double> d_all(2 * (size_t)k + 2 * (size_t)nthr); // errors (k) | sorted (k) | thresholds, aucs
    double *d = d_all.p;
    double *d_sorted = d + k, *d_thr = d_sorted + k, *d_auc = d_thr + nthr;
    MP_HIP(hipMemcpyAsync(d, errors, sizeof(double) * k, hipMemcpyHostToDevice, s));
    MP_HIP(hipMemcpyAsync(d_thr, thr, sizeof(double) * nthr, hipMemcpyHostToDevice, s));
    MP_HIP(launch_pose_auc(s, k, d, d_sorted, nthr, d_thr, d_auc));
    MP_HIP(hipMemcpyAsync(aucs, d_auc, sizeof(double) * nthr, hipMemcpyDeviceToHost, s));
    MP_HIP(hipStreamSynchronize(s));
}

void get_depths_batch(int dtype, int32_t num, const void *maps, const int64_t *dims, const int64_t *pt_off,
                      const double *pts, void *out, int device) {
    if (dtype != 0 && dtype != 1) throw std::invalid_argument("dtype must be 0 (float32) or 1 (float64)");
    if (num <= 0) return;
    const size_t es = dtype == 0 ? sizeof(float) : sizeof(double);
    std::vector<int64_t> map_off(num + 1), hw(2 * (size_t)num);
    std::vector<double> fac(2 * (size_t)num);
    map_off[0] = 0;
    for (int p = 0; p < num; ++p) {
        const int64_t h = dims[4 * p], w = dims[4 * p + 1], ih = dims[4 * p + 2], iw = dims[4 * p + 3];
        if (h <= 0 || w <= 0 || ih <= 0 || iw <= 0) throw std::invalid_argument("bad depth-map or image size");
        if (pt_off[p + 1] < pt_off[p]) throw std::invalid_argument("keypoint offsets must not decrease");
        map_off[p + 1] = map_off[p] + h * w;
        hw[2 * p] = h;
        hw[2 * p + 1] = w;
        fac[2 * p] = (double)w / (double)iw; // factor = [dm_w / im_w, dm_h / im_h]
        fac[2 * p + 1] = (double)h / (double)ih;
    }
    const int64_t total = pt_off[num], cells = map_off[num];
    CtxLease lease(device);
    hipStream_t s = lease.c->stream;
    DevArray<char> d_maps_a(es * (size_t)std::max<int64_t>(cells, 1)), d_out_a(es * (size_t)std::max<int64_t>(total, 1));
    DevArray<int64_t> d_map_off_a(num + 1), d_hw_a(2 * (size_t)num), d_pt_off_a(num + 1);
    DevArray<double> d_fac_a(2 * (size_t)num), d_pts_a(2 * (size_t)std::max<int64_t>(total, 1));
    char *d_maps = d_maps_a.p, *d_out = d_out_a.p;
    int64_t *d_map_off = d_map_off_a.p, *d_hw = d_hw_a.p, *d_pt_off = d_pt_off_a.p;
    double *d_fac = d_fac_a.p, *d_pts = d_pts_a.p;
    MP_HIP(hipMemcpyAsync(d_maps, maps, es * (size_t)cells, hipMemcpyHostToDevice, s));
    MP_HIP(hipMemcpyAsync(d_map_off, map_off.data(), sizeof(int64_t) * (num + 1), hipMemcpyHostToDevice, s));
    MP_HIP(hipMemcpyAsync(d_hw, hw.data(), sizeof(int64_t) * 2 * num, hipMemcpyHostToDevice, s));
    MP_HIP(hipMemcpyAsync(d_pt_off, pt_off, sizeof(int64_t) * (num + 1), hipMemcpyHostToDevice, s));
    MP_HIP(hipMemcpyAsync(d_fac, fac.data(), sizeof(double) * 2 * num, hipMemcpyHostToDevice, s));
    if (total > 0) MP_HIP(hipMemcpyAsync(d_pts, pts, sizeof(double) * 2 * total, hipMemcpyHostToDevice, s));
    MP_HIP(launch_get_depths(s, dtype, d_maps, d_map_off, d_hw, d_fac, d_pt_off, num, total, d_pts, d_out));
    if (total > 0) MP_HIP(hipMemcpyAsync(out, d_out, es * (size_t)total, hipMemcpyDeviceToHost, s));
    MP_HIP(hipStreamSynchronize(s));
}

void scale_and_pose_direct(const double *X, const double *Y, const double *W, int64_t n, Model *out, int device) {
    CtxLease lease(device);
    DeviceCtx &C = *lease.c;
    std::vector<double> in(7 * (size_t)n);
    std::memcpy(in.data(), X, sizeof(double) * 3 * n);
    std::memcpy(in.data() + 3 * n, Y, sizeof(double) * 3 * n);
    std::memcpy(in.data() + 6 * n, W, sizeof(double) * n);
    DevArray<double> d_in(in.size());
    DevArray<Model> d_out(1);
    MP_HIP(hipMemcpyAsync(d_in.p, in.data(), sizeof(double) * in.size(), hipMemcpyHostToDevice, C.stream));
    MP_HIP(launch_scale_and_pose(C.stream, d_in.p, n, d_out.p));
    MP_HIP(hipMemcpyAsync(out, d_out.p, sizeof(Model), hipMemcpyDeviceToHost, C.stream));
    MP_HIP(hipStreamSynchronize(C.stream));
}

int device_count() {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess) return 0;
    return cnt;
}

} // namespace mp
