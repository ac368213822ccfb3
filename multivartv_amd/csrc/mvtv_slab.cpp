// mvtv_slab.cpp — one mesh decomposed over ranks (SURVEY §8e, config 5 / the metric at 2-8 GPUs): the whole
// variant-B ADMM loop (rcpp-code/MultivarTV/src/solvers.cpp:110-133) of one rank, enqueued on the problem's
// stream with its collectives, decided on the device, polled by the host only every few iterations.
//
// Rank r owns planes [zb, ze) of the last dimension plus one ghost plane below / above
// (mvtv_problem_create_slab). Per iteration:
//   theta-solve  cosine transforms along dims 0..p-2 on the owned planes, in place; the tridiagonal line
//                solves along dim p-1 by substructuring (mvtv_spectral.hip k_tris): each rank reduces its
//                block of every line to 6 numbers, an all-to-all brings each chunk of lines' numbers to
//                one rank, which solves the lines' interface systems over the ranks and sends every rank
//                its lines' 2 neighbour values back; each rank then solves its blocks; inverse transforms
//                along dims p-2..0 in place. 8 numbers per line cross the ranks instead of the mesh twice.
//   theta halo   first owned plane -> rank-1's upper ghost, last -> rank+1's lower ghost.
//   edge update  p = 3: the fused pass (k_admm3a) on the owned planes: its chunk-start recompute of
//   + gather     plane zb-1 reads theta's lower ghost and z_old's lower ghost plane, which rank-1 sent
//                at the end of the previous iteration; p = 4: edge update, z lower-ghost halo, gather.
//   reductions   one all-reduce of the 7 partial sums into the device control block; k_admm_control
//                then takes adapt_step / stopping on every rank from bit-identical inputs.
//   z halo       (p = 3) last owned plane of z_new -> rank+1's ghost plane of the same buffer.
// The collectives run on a stream of their own, handed their inputs by events, so the z halo overlaps the
// next iteration's theta-solve. Transports (mvtv_comm): RCCL over xGMI (one process per GPU; ROCm's
// librccl.so.1 is dlopen'd at the first communicator, never torch's copy: see rccl_api) or an in-process
// loopback group (every rank on its own host thread, device-to-device copies between the ranks' buffers):
// the same loop, testable on one GPU.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "mvtv_problem.h"

// ============================================================================================ transports
struct mvtv_comm {
    int rank = 0, size = 1;
    int device = 0;                  // RCCL: the communicator's device
    double* scratch = nullptr;       // mvtv_comm_allreduce_host's device staging (RCCL)
    hipStream_t stream = nullptr;
    virtual ~mvtv_comm() = default;
    // point-to-point transfers between begin() and end() progress together (all-to-all, halos)
    virtual mvtv_status begin() = 0;
    virtual mvtv_status send(const double* buf, size_t n, int peer, hipStream_t s) = 0;
    virtual mvtv_status recv(double* buf, size_t n, int peer, hipStream_t s) = 0;
    virtual mvtv_status end(hipStream_t s) = 0;
    virtual mvtv_status allreduce_sum(double* buf, size_t n, hipStream_t s) = 0;
    // a rank whose loop failed tells its peers, so that they fail instead of waiting for it (loopback, ipc; an
    // RCCL peer of a failed process is ended by the launcher)
    virtual void abort() {}
    // called at the start of every mvtv_slab_run (the ipc transport drops its buffer mappings there; RCCL splits off
    // its second communicator there, a collective call every rank makes at the same point); non-OK: no second lane
    virtual mvtv_status run_begin() { return MVTV_OK; }
    // lanes: independent orderings of collectives, so the critical-path collectives (lane 0, issued on the compute
    // stream) and the halos (lane 1, on the collectives stream) may run concurrently. RCCL: one communicator per
    // lane (two ops of one communicator must not run at once on different streams); the loopback and ipc groups match
    // their transfers in host program order, which every rank shares, so both lanes are the same group there
    virtual int lanes() const { return 2; }
    virtual void set_lane(int) {}
};

namespace {

// ---- RCCL, resolved with dlopen ------------------------------------------------------------------
struct RcclApi {
    void* h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) = nullptr;
    std::string path;   // the file the functions came from
};

mvtv_status rccl_api(RcclApi** out) {
    static RcclApi api;
    static bool tried = false;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (!tried) {
        tried = true;
        // ROCm's librccl, which shares libmvtv's HIP runtime (/opt/rocm). A librccl that `import torch` maps
        // is NOT reused: torch's links torch's own copy of the HIP runtime, on which libmvtv's streams are
        // invalid ("unhandled cuda error" at ncclCommInitRank). Callers keep one RCCL *running* per process
        // by giving torch.distributed the gloo backend (bench.py), so torch's copy is never initialised.
        for (const char* name : {"/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"}) {
            api.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (api.h) break;
        }
        if (api.h) {
            auto sym = [&](auto& fp, const char* n) { fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(api.h, n)); };
            sym(api.GetUniqueId, "ncclGetUniqueId");
            sym(api.CommInitRank, "ncclCommInitRank");
            sym(api.CommDestroy, "ncclCommDestroy");
            sym(api.Send, "ncclSend");
            sym(api.Recv, "ncclRecv");
            sym(api.GroupStart, "ncclGroupStart");
            sym(api.GroupEnd, "ncclGroupEnd");
            sym(api.AllReduce, "ncclAllReduce");
            sym(api.GetErrorString, "ncclGetErrorString");
            sym(api.CommSplit, "ncclCommSplit");
            Dl_info info{};
            if (api.GetUniqueId && dladdr(reinterpret_cast<void*>(api.GetUniqueId), &info) && info.dli_fname)
                api.path = info.dli_fname;
        }
    }
    if (!api.h || !api.GetUniqueId || !api.CommInitRank || !api.Send || !api.Recv || !api.GroupStart ||
        !api.GroupEnd || !api.AllReduce)
        return fail(MVTV_HIP_ERROR, "RCCL (librccl.so.1) not available");
    *out = &api;
    return MVTV_OK;
}

#define NCCL_TRY(expr)                                                                              \
    do {                                                                                            \
        ncclResult_t _r = (expr);                                                                   \
        if (_r != ncclSuccess)                                                                      \
            return fail(MVTV_HIP_ERROR, std::string("RCCL: ") + #expr + ": " +                     \
                                            (api_->GetErrorString ? api_->GetErrorString(_r) : "?")); \
    } while (0)

// a transfer to / from this rank itself is a device copy: sends are stashed, the matching recv copies
struct SelfCopy {
    std::deque<std::pair<const double*, size_t>> q;
    mvtv_status recv(double* buf, size_t n, hipStream_t s) {
        if (q.empty() || q.front().second != n) return fail(MVTV_BAD_ARG, "self transfer without its send");
        HIP_TRY(hipMemcpyAsync(buf, q.front().first, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        q.pop_front();
        return MVTV_OK;
    }
};

// Every transfer goes through RCCL, the rank's own ones too (send / recv to self in the group), and the
// all-reduce runs at one rank as well: one-GPU runs of the distributed loop (MVTV_SLAB_DISTRIBUTED=1 at
// world size 1) execute the same RCCL calls as the 8-GPU runs.
struct RcclComm final : mvtv_comm {
    RcclApi* api_ = nullptr;
    ncclComm_t comm = nullptr;
    ncclComm_t comm2 = nullptr;   // lane 1 (the halos), split off comm at the first run
    bool split_tried = false;
    int lane_ = 0;
    ncclComm_t cur() const { return lane_ == 1 && comm2 ? comm2 : comm; }
    mvtv_status run_begin() override {
        lane_ = 0;
        if (!split_tried) {   // every rank reaches this at its first run: a collective call in the same order
            split_tried = true;
            // The second lane is opt-in (MVTV_RCCL_SPLIT=1) until a multi-GPU RCCL run has exercised it; with it on,
            // the ranks agree on the outcome before any rank uses it: one rank on comm2 while its peers stay on comm
            // would post mismatched operations and hang inside the loop
            const char* e = std::getenv("MVTV_RCCL_SPLIT");
            if (e && std::atoi(e) != 0) {
                DeviceGuard dg(device);
                bool ok = api_->CommSplit && api_->CommSplit(comm, 0, rank, &comm2, nullptr) == ncclSuccess;
                if (!ok) comm2 = nullptr;
                double host[1] = {ok ? 0.0 : 1.0};
                bool agreed = false;
                if (stream || hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess) {
                    if (scratch || alloc(&scratch, 64) == MVTV_OK) {
                        agreed = hipMemcpyAsync(scratch, host, sizeof(double), hipMemcpyHostToDevice, stream) == hipSuccess &&
                                 api_->AllReduce(scratch, scratch, 1, ncclFloat64, ncclSum, comm, stream) == ncclSuccess &&
                                 hipMemcpyAsync(host, scratch, sizeof(double), hipMemcpyDeviceToHost, stream) == hipSuccess &&
                                 hipStreamSynchronize(stream) == hipSuccess;
                    }
                }
                if (!agreed || host[0] != 0.0) {   // some rank has no second communicator: every rank keeps one lane
                    if (comm2 && api_->CommDestroy) api_->CommDestroy(comm2);
                    comm2 = nullptr;
                    (void)hipGetLastError();
                    std::fprintf(stderr, "mvtv: RCCL second lane not on every rank (%g failed); one lane\n", host[0]);
                }
            }
        }
        return MVTV_OK;
    }
    int lanes() const override { return comm2 ? 2 : 1; }
    void set_lane(int l) override { lane_ = l; }
    ~RcclComm() override {
        if (comm2 && api_->CommDestroy) api_->CommDestroy(comm2);
        if (comm && api_->CommDestroy) api_->CommDestroy(comm);
        if (scratch) (void)hipFree(scratch);
        if (stream) (void)hipStreamDestroy(stream);
    }
    mvtv_status begin() override {
        NCCL_TRY(api_->GroupStart());
        return MVTV_OK;
    }
    mvtv_status send(const double* buf, size_t n, int peer, hipStream_t s) override {
        NCCL_TRY(api_->Send(buf, n, ncclFloat64, peer, cur(), s));
        return MVTV_OK;
    }
    mvtv_status recv(double* buf, size_t n, int peer, hipStream_t s) override {
        NCCL_TRY(api_->Recv(buf, n, ncclFloat64, peer, cur(), s));
        return MVTV_OK;
    }
    mvtv_status end(hipStream_t) override {
        NCCL_TRY(api_->GroupEnd());
        return MVTV_OK;
    }
    mvtv_status allreduce_sum(double* buf, size_t n, hipStream_t s) override {
        NCCL_TRY(api_->AllReduce(buf, buf, n, ncclFloat64, ncclSum, cur(), s));
        return MVTV_OK;
    }
};

// ---- in-process loopback group --------------------------------------------------------------------
// Every rank runs its loop on its own host thread; a transfer is a device-to-device copy enqueued by the
// receiver after the sender's data-ready event, and the sender's stream waits for the copy's event before
// it goes on (so it cannot overwrite the source early). The all-reduce copies every rank's vector into
// each rank's staging rows and sums them in rank order, so all ranks get bit-identical sums.
struct LocalHub {
    int size = 0;
    std::mutex mu;
    std::condition_variable cv;
    struct Msg {
        const double* src;
        size_t n;
        hipEvent_t ready;   // sender's data is complete
        hipEvent_t* done;   // receiver records its copy's completion here
        bool* acked;
    };
    std::vector<std::deque<Msg>> box;   // box[from * size + to]
    // all-reduce rendezvous
    int arrive = 0, leave = 0;
    long gen = 0;
    std::vector<double*> bufs;
    std::vector<hipEvent_t> bev, cev;
    std::vector<hipEvent_t> pool;   // events of finished transfers, reused (guarded by mu)
    bool aborted = false;           // some rank's loop failed: every wait gives up
    explicit LocalHub(int g) : size(g), box(size_t(g) * size_t(g)), bufs(size_t(g)), bev(size_t(g)), cev(size_t(g)) {}
    ~LocalHub() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
    hipEvent_t event() {   // call with mu held
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        return e;
    }
};

__global__ void k_rowsum(const double* __restrict__ stage, int rows, int n, double* __restrict__ out) {
    const int i = int(threadIdx.x);
    if (i >= n) return;
    double acc = 0.0;
    for (int r = 0; r < rows; ++r) acc += stage[r * n + i];
    out[i] = acc;
}

struct LocalComm final : mvtv_comm {
    std::shared_ptr<LocalHub> hub;
    struct Pending {
        hipEvent_t ready;   // our data-ready event (recycled once the receiver has waited on it)
        hipEvent_t done;    // the receiver's copy-complete event
        bool acked;
    };
    std::deque<Pending> sent;   // this group's sends (stable addresses)
    double* stage = nullptr;
    size_t stage_n = 0;
    SelfCopy self;
    ~LocalComm() override {
        if (stage) (void)hipFree(stage);
    }
    hipEvent_t event() {
        std::lock_guard<std::mutex> lk(hub->mu);
        return hub->event();
    }
    mvtv_status begin() override {
        sent.clear();
        return MVTV_OK;
    }
    mvtv_status send(const double* buf, size_t n, int peer, hipStream_t s) override {
        if (peer == rank) {
            self.q.emplace_back(buf, n);
            return MVTV_OK;
        }
        hipEvent_t ready = event();
        HIP_TRY(hipEventRecord(ready, s));
        sent.push_back(Pending{ready, nullptr, false});
        Pending& pd = sent.back();
        std::lock_guard<std::mutex> lk(hub->mu);
        hub->box[size_t(rank) * size_t(size) + size_t(peer)].push_back(LocalHub::Msg{buf, n, ready, &pd.done, &pd.acked});
        hub->cv.notify_all();
        return MVTV_OK;
    }
    mvtv_status recv(double* buf, size_t n, int peer, hipStream_t s) override {
        if (peer == rank) return self.recv(buf, n, s);
        LocalHub::Msg m{};
        {
            std::unique_lock<std::mutex> lk(hub->mu);
            auto& q = hub->box[size_t(peer) * size_t(size) + size_t(rank)];
            hub->cv.wait(lk, [&] { return !q.empty() || hub->aborted; });
            if (q.empty()) return fail(MVTV_HIP_ERROR, "loopback: a peer rank aborted");
            m = q.front();
            q.pop_front();
        }
        if (m.n != n) return fail(MVTV_BAD_ARG, "loopback transfer size mismatch");
        HIP_TRY(hipStreamWaitEvent(s, m.ready, 0));
        HIP_TRY(hipMemcpyAsync(buf, m.src, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        hipEvent_t done = event();
        HIP_TRY(hipEventRecord(done, s));
        std::lock_guard<std::mutex> lk(hub->mu);
        *m.done = done;
        *m.acked = true;
        hub->cv.notify_all();
        return MVTV_OK;
    }
    mvtv_status end(hipStream_t s) override {
        std::unique_lock<std::mutex> lk(hub->mu);
        hub->cv.wait(lk, [&] {
            if (hub->aborted) return true;
            for (auto& pd : sent)
                if (!pd.acked) return false;
            return true;
        });
        if (hub->aborted) return fail(MVTV_HIP_ERROR, "loopback: a peer rank aborted");
        lk.unlock();
        for (auto& pd : sent) HIP_TRY(hipStreamWaitEvent(s, pd.done, 0));
        lk.lock();   // both events have been waited on by the streams that need them: reusable
        for (auto& pd : sent) {
            hub->pool.push_back(pd.ready);
            hub->pool.push_back(pd.done);
        }
        sent.clear();
        return MVTV_OK;
    }
    // generation barrier on the hub; false when a peer aborted
    bool barrier(std::unique_lock<std::mutex>& lk) {
        if (hub->aborted) return false;
        const long g = hub->gen;
        if (++hub->arrive == size) {
            hub->arrive = 0;
            ++hub->gen;
            hub->cv.notify_all();
        } else {
            hub->cv.wait(lk, [&] { return hub->gen != g || hub->aborted; });
        }
        return hub->gen != g;
    }
    void abort() override {
        std::lock_guard<std::mutex> lk(hub->mu);
        hub->aborted = true;
        hub->cv.notify_all();
    }
    mvtv_status allreduce_sum(double* buf, size_t n, hipStream_t s) override {
        if (size == 1) return MVTV_OK;
        if (n > 64) return fail(MVTV_BAD_ARG, "loopback all-reduce of more than 64 values");
        if (stage_n < n * size_t(size)) {
            if (stage) (void)hipFree(stage);
            stage = nullptr;
            MVTV_TRY(alloc(&stage, n * size_t(size)));
            stage_n = n * size_t(size);
        }
        hipEvent_t ready = event(), copied = event();
        HIP_TRY(hipEventRecord(ready, s));
        std::unique_lock<std::mutex> lk(hub->mu);
        hub->bufs[size_t(rank)] = buf;
        hub->bev[size_t(rank)] = ready;
        if (!barrier(lk)) return fail(MVTV_HIP_ERROR, "loopback: a peer rank aborted");   // every vector posted
        lk.unlock();
        for (int r = 0; r < size; ++r) {
            HIP_TRY(hipStreamWaitEvent(s, hub->bev[size_t(r)], 0));
            HIP_TRY(hipMemcpyAsync(stage + size_t(r) * n, hub->bufs[size_t(r)], n * sizeof(double),
                                   hipMemcpyDeviceToDevice, s));
        }
        HIP_TRY(hipEventRecord(copied, s));
        lk.lock();
        hub->cev[size_t(rank)] = copied;
        if (!barrier(lk)) return fail(MVTV_HIP_ERROR, "loopback: a peer rank aborted");   // copies enqueued
        lk.unlock();
        for (int r = 0; r < size; ++r)   // nobody overwrites its vector before all copies of it are done
            if (r != rank) HIP_TRY(hipStreamWaitEvent(s, hub->cev[size_t(r)], 0));
        hipLaunchKernelGGL(k_rowsum, dim3(1), dim3(64), 0, s, stage, size, int(n), buf);
        HIP_TRY(hipGetLastError());
        lk.lock();
        if (!barrier(lk)) return fail(MVTV_HIP_ERROR, "loopback: a peer rank aborted");   // slots reusable
        hub->pool.push_back(ready);
        hub->pool.push_back(copied);
        lk.unlock();
        return MVTV_OK;
    }
};

// ---- inter-process group over HIP IPC memory --------------------------------------------------------------
// One process per rank, the ranks' devices the same GPU or peers on one node. Data moves device to device: the
// sender copies a group's send buffers into its own staging buffer (one allocation, grown when a group needs more)
// and the receiver copies out of it, mapped once with hipIpcOpenMemHandle (same GPU: HBM copies; peer GPUs: a P2P
// read over xGMI). Staging instead of mapping the problem's own buffers: importing an 8 GB edge-state allocation
// (a 128^4 rank's) never returned on the box, while the staging buffer holds only a message group (<= a few
// hundred MB: a 4-D rank's z plane). Ordering goes through the host: a rendezvous segment in POSIX shared
// memory holds, per (sender, receiver) channel, a ring of posted messages (staging handle and generation,
// offset, count) and post / ack counters; the all-reduce is a rank-ordered host sum of every rank's staged vector (bit-identical on
// every rank, as the loopback's). end() is where a group's transfers happen: the sender waits for its data
// (its stream), posts every send, the receiver copies every posted buffer it expects, waits for the copies and
// acks, and the sender returns once its peers have acked, so nothing enqueued after end() can overwrite a
// source before it was read. The host waits inside a collective, so the z halo does not overlap the next
// theta-solve as it does under RCCL: this transport is for correctness of the multi-process path (and a
// fallback when RCCL has no communicator), not the tuned one. Every wait polls the segment's abort flag and
// gives up after MVTV_IPC_TIMEOUT seconds (default 300), so a dead peer ends the others with an error.
constexpr int IPC_MAX_RANKS = 16;
constexpr int IPC_RING = 64;
constexpr uint64_t IPC_MAGIC = 0x4d5654564950430aull;

struct IpcSlot {
    hipIpcMemHandle_t handle;   // the sender's staging buffer
    uint64_t gen;               // its allocation generation (the receiver re-maps when it changes)
    uint64_t offset, n;
};
struct IpcChan {
    std::atomic<uint64_t> posted;
    std::atomic<uint64_t> acked;
    IpcSlot slot[IPC_RING];
};
struct IpcShm {
    std::atomic<uint64_t> magic;
    std::atomic<int32_t> size;
    std::atomic<int32_t> attached;
    std::atomic<int32_t> aborted;
    std::atomic<uint64_t> barrier;   // monotone arrival count: the k-th barrier ends at size * k
    double ar[IPC_MAX_RANKS][64];
    IpcChan ch[IPC_MAX_RANKS * IPC_MAX_RANKS];
};

struct IpcComm final : mvtv_comm {
    IpcShm* shm = nullptr;
    std::string name;
    uint64_t nbar = 0;                              // barriers this rank has passed
    std::vector<uint64_t> sent_n, recv_n;           // per peer: messages posted to / consumed from
    struct Out { const double* buf; size_t n; int peer; };
    struct In { double* buf; size_t n; int peer; };
    std::vector<Out> outs;
    std::vector<In> ins;
    SelfCopy self;
    double* stage = nullptr;                        // this rank's staging buffer (exported)
    size_t stage_words = 0;
    uint64_t stage_gen = 0;
    hipIpcMemHandle_t stage_handle{};
    struct Mapped { uint64_t gen = 0; char* ptr = nullptr; };
    std::vector<Mapped> mapped;                     // per peer: its staging buffer in this process
    double timeout_s = 300.0;
    bool trace = false;                                                 // MVTV_IPC_TRACE=1: every step to stderr
    long ncoll = 0;
    void tr(const char* what, long a = -1, long b = -1) const {
        if (!trace) return;
        const double ts = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        std::fprintf(stderr, "[ipc %d %.6f] #%ld %s %ld %ld\n", rank, ts, ncoll, what, a, b);
        std::fflush(stderr);
    }

    ~IpcComm() override {
        close_mappings();
        if (stage) {
            DeviceGuard dg(device);
            (void)hipFree(stage);
        }
        if (shm) munmap(shm, sizeof(IpcShm));
    }
    void close_mappings() {
        // no HIP call (and no runtime initialisation) when nothing is mapped: the host-only transport tests
        const bool any = std::any_of(mapped.begin(), mapped.end(), [](const Mapped& mp) { return mp.ptr != nullptr; });
        if (any) {
            DeviceGuard dg(device);
            for (auto& mp : mapped)
                if (mp.ptr) (void)hipIpcCloseMemHandle(mp.ptr);
        }
        mapped.assign(size_t(size), Mapped{});
    }
    void abort() override {
        if (shm) shm->aborted.store(1);
    }
    mvtv_status run_begin() override {
        close_mappings();
        return MVTV_OK;
    }
    // poll until pred() holds; false on abort or timeout
    template <class F>
    bool wait(F pred, const char* what, mvtv_status* st) {
        const auto t0 = std::chrono::steady_clock::now();
        for (long spin = 0;; ++spin) {
            if (pred()) return true;
            if (shm->aborted.load()) {
                *st = fail(MVTV_HIP_ERROR, std::string("ipc transport: a peer rank aborted (") + what + ")");
                return false;
            }
            if (spin > 2000) {
                std::this_thread::sleep_for(std::chrono::microseconds(20));
                if ((spin & 1023) == 0 &&
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
                    shm->aborted.store(1);
                    *st = fail(MVTV_HIP_ERROR, std::string("ipc transport: timed out waiting for ") + what);
                    return false;
                }
            }
        }
    }
    mvtv_status host_barrier(const char* what) {
        ++nbar;
        shm->barrier.fetch_add(1);
        mvtv_status st = MVTV_OK;
        const uint64_t target = nbar * uint64_t(size);
        if (!wait([&] { return shm->barrier.load() >= target; }, what, &st)) return st;
        return MVTV_OK;
    }
    mvtv_status begin() override {
        outs.clear();
        ins.clear();
        return MVTV_OK;
    }
    mvtv_status send(const double* buf, size_t n, int peer, hipStream_t) override {
        if (peer == rank) {
            self.q.emplace_back(buf, n);
            return MVTV_OK;
        }
        outs.push_back(Out{buf, n, peer});
        return MVTV_OK;
    }
    mvtv_status recv(double* buf, size_t n, int peer, hipStream_t s) override {
        if (peer == rank) return self.recv(buf, n, s);   // enqueued now: in order on s, before end()'s copies
        ins.push_back(In{buf, n, peer});
        return MVTV_OK;
    }
    mvtv_status end(hipStream_t s) override {
        DeviceGuard dg(device);
        mvtv_status st = MVTV_OK;
        ++ncoll;
        tr("end: sends / recvs", long(outs.size()), long(ins.size()));
        // the group's sends into the staging buffer (each message 256-B aligned), grown if the group needs more
        std::vector<size_t> off(outs.size());
        size_t words = 0;
        for (size_t i = 0; i < outs.size(); ++i) {
            off[i] = words;
            words += (outs[i].n + 31) / 32 * 32;
        }
        if (words > stage_words) {
            if (stage) HIP_TRY(hipFree(stage));
            stage = nullptr;
            stage_words = std::max<size_t>(words, size_t(1) << 20);
            MVTV_TRY(alloc(&stage, stage_words));
            HIP_TRY(hipIpcGetMemHandle(&stage_handle, stage));
            ++stage_gen;
            tr("end: staging (MB)", long((stage_words * 8) >> 20));
        }
        for (size_t i = 0; i < outs.size(); ++i)
            HIP_TRY(hipMemcpyAsync(stage + off[i], outs[i].buf, outs[i].n * sizeof(double), hipMemcpyDeviceToDevice, s));
        if (!outs.empty()) HIP_TRY(hipStreamSynchronize(s));   // every send's data is staged
        tr("end: data ready");
        for (size_t i = 0; i < outs.size(); ++i) {
            const Out& o = outs[i];
            IpcChan& c = shm->ch[rank * IPC_MAX_RANKS + o.peer];
            const uint64_t k = sent_n[size_t(o.peer)];
            if (!wait([&] { return k - c.acked.load() < uint64_t(IPC_RING); }, "a free ring slot", &st)) return st;
            IpcSlot& sl = c.slot[k % IPC_RING];
            sl.handle = stage_handle;
            sl.gen = stage_gen;
            sl.offset = uint64_t(off[i]) * sizeof(double);
            sl.n = o.n;
            c.posted.store(k + 1);   // release: the slot's contents before the count
            sent_n[size_t(o.peer)] = k + 1;
        }
        for (const In& i : ins) {
            IpcChan& c = shm->ch[i.peer * IPC_MAX_RANKS + rank];
            const uint64_t k = recv_n[size_t(i.peer)];
            if (!wait([&] { return c.posted.load() > k; }, "a peer's send", &st)) return st;
            const IpcSlot& sl = c.slot[k % IPC_RING];
            if (sl.n != i.n) return fail(MVTV_BAD_ARG, "ipc transfer size mismatch");
            Mapped& mp = mapped[size_t(i.peer)];
            if (!mp.ptr || mp.gen != sl.gen) {   // the peer's (new) staging buffer
                if (mp.ptr) HIP_TRY(hipIpcCloseMemHandle(mp.ptr));
                mp.ptr = nullptr;
                void* p = nullptr;
                tr("end: open peer staging", i.peer, long(sl.gen));
                HIP_TRY(hipIpcOpenMemHandle(&p, sl.handle, hipIpcMemLazyEnablePeerAccess));
                tr("end: opened");
                mp.ptr = static_cast<char*>(p);
                mp.gen = sl.gen;
            }
            tr("end: copy from peer", i.peer, long(i.n));
            HIP_TRY(hipMemcpyAsync(i.buf, mp.ptr + sl.offset, i.n * sizeof(double), hipMemcpyDeviceToDevice, s));
        }
        if (!ins.empty()) HIP_TRY(hipStreamSynchronize(s));   // the copies have read their sources
        tr("end: copies done");
        for (const In& i : ins) {
            IpcChan& c = shm->ch[i.peer * IPC_MAX_RANKS + rank];
            recv_n[size_t(i.peer)] += 1;
            c.acked.store(recv_n[size_t(i.peer)]);
        }
        for (const Out& o : outs) {
            IpcChan& c = shm->ch[rank * IPC_MAX_RANKS + o.peer];
            const uint64_t k = sent_n[size_t(o.peer)];
            if (!wait([&] { return c.acked.load() >= k; }, "a peer's ack", &st)) return st;
        }
        tr("end: acked");
        outs.clear();
        ins.clear();
        return MVTV_OK;
    }
    mvtv_status allreduce_host_vals(double* v, size_t n) {
        if (n > 64) return fail(MVTV_BAD_ARG, "ipc all-reduce of more than 64 values");
        std::memcpy(shm->ar[rank], v, n * sizeof(double));
        MVTV_TRY(host_barrier("the all-reduce"));          // every vector posted
        for (size_t i = 0; i < n; ++i) {
            double acc = 0.0;
            for (int r = 0; r < size; ++r) acc += shm->ar[r][i];
            v[i] = acc;
        }
        return host_barrier("the all-reduce");             // slots reusable
    }
    mvtv_status allreduce_sum(double* buf, size_t n, hipStream_t s) override {
        if (size == 1) return MVTV_OK;
        DeviceGuard dg(device);
        double v[64];
        if (n > 64) return fail(MVTV_BAD_ARG, "ipc all-reduce of more than 64 values");
        ++ncoll;
        tr("allreduce", long(n));
        HIP_TRY(hipMemcpyAsync(v, buf, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        tr("allreduce: staged");
        MVTV_TRY(allreduce_host_vals(v, n));
        HIP_TRY(hipMemcpyAsync(buf, v, n * sizeof(double), hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
        return MVTV_OK;
    }
};

}  // namespace

// ============================================================================================ C ABI
extern "C" {

mvtv_status mvtv_comm_unique_id(uint8_t* out128) {
    if (!out128) return fail(MVTV_BAD_ARG, "null argument");
    RcclApi* api = nullptr;
    MVTV_TRY(rccl_api(&api));
    ncclUniqueId id;
    if (api->GetUniqueId(&id) != ncclSuccess) return fail(MVTV_HIP_ERROR, "ncclGetUniqueId failed");
    std::memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return MVTV_OK;
}

mvtv_status mvtv_comm_create_rccl(const uint8_t* id128, int32_t nranks, int32_t rank, int32_t device,
                                  mvtv_comm** out) {
    if (!id128 || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(MVTV_BAD_ARG, "bad argument");
    RcclApi* api = nullptr;
    MVTV_TRY(rccl_api(&api));
    DeviceGuard dg(device);
    auto* c = new RcclComm();
    c->api_ = api;
    c->rank = rank;
    c->size = nranks;
    c->device = device;
    ncclUniqueId id;
    std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = api->CommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        delete c;
        return fail(MVTV_HIP_ERROR, std::string("ncclCommInitRank: ") + (api->GetErrorString ? api->GetErrorString(r) : "?"));
    }
    *out = c;
    return MVTV_OK;
}

mvtv_status mvtv_comm_create_local(int32_t nranks, mvtv_comm** out) {
    if (!out || nranks < 1 || nranks > 64) return fail(MVTV_BAD_ARG, "nranks must be 1..64");
    auto hub = std::make_shared<LocalHub>(nranks);
    for (int r = 0; r < nranks; ++r) {
        auto* c = new LocalComm();
        c->hub = hub;
        c->rank = r;
        c->size = nranks;
        out[r] = c;
    }
    return MVTV_OK;
}

mvtv_status mvtv_comm_create_ipc(const char* name, int32_t nranks, int32_t rank, int32_t device, mvtv_comm** out) {
    if (!name || !out || name[0] != '/' || nranks < 1 || nranks > IPC_MAX_RANKS || rank < 0 || rank >= nranks)
        return fail(MVTV_BAD_ARG, "bad argument (name '/...', 1 <= nranks <= 16)");
    auto c = std::make_unique<IpcComm>();
    c->rank = rank;
    c->size = nranks;
    c->device = device;
    c->name = name;
    c->sent_n.assign(size_t(nranks), 0);
    c->recv_n.assign(size_t(nranks), 0);
    c->mapped.assign(size_t(nranks), IpcComm::Mapped{});
    if (const char* t = std::getenv("MVTV_IPC_TIMEOUT")) c->timeout_s = std::max(1.0, std::atof(t));
    if (const char* t = std::getenv("MVTV_IPC_TRACE")) c->trace = std::atoi(t) != 0;
    const size_t bytes = sizeof(IpcShm);
    int fd = -1;
    const auto t0 = std::chrono::steady_clock::now();
    auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    if (rank == 0) {
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) return fail(MVTV_HIP_ERROR, std::string("ipc transport: shm_open(create) ") + name + ": " + std::strerror(errno));
        if (ftruncate(fd, off_t(bytes)) != 0) {
            close(fd);
            shm_unlink(name);
            return fail(MVTV_HIP_ERROR, "ipc transport: ftruncate failed");
        }
    } else {
        while ((fd = shm_open(name, O_RDWR, 0600)) < 0) {   // rank 0 creates it
            if (elapsed() > c->timeout_s) return fail(MVTV_HIP_ERROR, std::string("ipc transport: no segment ") + name);
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
        struct stat sb {};
        while (fstat(fd, &sb) == 0 && size_t(sb.st_size) < bytes) {
            if (elapsed() > c->timeout_s) {
                close(fd);
                return fail(MVTV_HIP_ERROR, "ipc transport: segment never sized");
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        if (rank == 0) shm_unlink(name);
        return fail(MVTV_HIP_ERROR, "ipc transport: mmap failed");
    }
    c->shm = static_cast<IpcShm*>(m);   // a fresh segment is zero-filled: every counter starts at 0
    if (rank == 0) {
        c->shm->size.store(nranks);
        c->shm->magic.store(IPC_MAGIC);
    } else {
        while (c->shm->magic.load() != IPC_MAGIC) {
            if (elapsed() > c->timeout_s) return fail(MVTV_HIP_ERROR, "ipc transport: segment never initialised");
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (c->shm->size.load() != nranks) return fail(MVTV_BAD_ARG, "ipc transport: rank count differs from rank 0's");
    }
    c->shm->attached.fetch_add(1);
    mvtv_status st = MVTV_OK;
    if (!c->wait([&] { return c->shm->attached.load() >= nranks; }, "every rank to attach", &st)) {
        if (rank == 0) shm_unlink(name);
        return st;
    }
    if (rank == 0) shm_unlink(name);   // every rank has it mapped: nothing is left in /dev/shm
    *out = c.release();
    return MVTV_OK;
}

void mvtv_comm_destroy(mvtv_comm* c) { delete c; }

mvtv_status mvtv_comm_allreduce_host(mvtv_comm* c, double* vals, int32_t n) {
    if (!c || (!vals && n > 0) || n < 0 || n > 64) return fail(MVTV_BAD_ARG, "bad argument (n <= 64)");
    if (n == 0) return MVTV_OK;
    if (auto* ic = dynamic_cast<IpcComm*>(c)) return ic->size == 1 ? MVTV_OK : ic->allreduce_host_vals(vals, size_t(n));
    if (!dynamic_cast<RcclComm*>(c)) return fail(MVTV_BAD_ARG, "host all-reduce: RCCL or ipc communicators only");
    c->set_lane(0);
    DeviceGuard dg(c->device);
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->scratch) MVTV_TRY(alloc(&c->scratch, 64));
    HIP_TRY(hipMemcpyAsync(c->scratch, vals, size_t(n) * sizeof(double), hipMemcpyHostToDevice, c->stream));
    MVTV_TRY(c->allreduce_sum(c->scratch, size_t(n), c->stream));
    HIP_TRY(hipMemcpyAsync(vals, c->scratch, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MVTV_OK;
}

const char* mvtv_comm_library(void) {
    RcclApi* api = nullptr;
    if (rccl_api(&api) != MVTV_OK) return "";
    return api->path.c_str();
}
int32_t mvtv_comm_rank(const mvtv_comm* c) { return c ? c->rank : -1; }
int32_t mvtv_comm_size(const mvtv_comm* c) { return c ? c->size : 0; }

}  // extern "C"

// ============================================================================================ the loop
namespace {

struct SlabGeom {
    uint32_t plane = 0, nz = 0, zb = 0, mg = 0, lines = 0, chunk = 0;
    size_t off = 0;   // first owned node
};

}  // namespace

namespace {
mvtv_status slab_run(mvtv_problem* P, mvtv_comm* C, const mvtv_admm_opts* opts, double lambda, double theta0,
                     double rho0, mvtv_admm_stats* stats) {
    if (!P->slab) return fail(MVTV_BAD_ARG, "not a slab problem (mvtv_problem_create_slab)");
    if (opts->variant != MVTV_VARIANT_RCPP) return fail(MVTV_BAD_ARG, "the slab loop runs variant B");
    if (P->wmode == W_NONE || !P->spec_lead || P->g.p < 2)
        return fail(MVTV_BAD_ARG, "slab loop: W = I or diagonal, p >= 2, m_j <= 4096 for j < p - 1");
    if (C->size == 1 && !P->spec_mesh)
        return fail(MVTV_BAD_ARG, "slab loop on one rank: the last dimension too must be <= 4096");
    if (!(lambda >= 0.0) || !(rho0 > 0.0)) return fail(MVTV_BAD_ARG, "lambda >= 0 and rho0 > 0");
    const auto t0 = std::chrono::steady_clock::now();
    DeviceGuard dg(P->device);
    const int p = P->g.p, G = C->size, rk = C->rank;
    hipStream_t s = P->stream;
    SlabGeom sg;
    sg.plane = P->g.N / P->g.m[p - 1];
    sg.nz = uint32_t(P->ze - P->zb);
    sg.zb = uint32_t(P->zb);
    sg.mg = uint32_t(P->m_global);
    sg.lines = sg.plane;
    sg.off = size_t(P->g_lo) * sg.plane;
    if (sg.lines % uint32_t(G) != 0) return fail(MVTV_BAD_ARG, "lines must split evenly over the ranks");
    sg.chunk = sg.lines / uint32_t(G);
    // every rank's plane range, floor(m_global r / G) as plane_bounds (multivartv_amd/slab.py): the
    // all-to-all counts
    std::vector<uint32_t> zbs(size_t(G) + 1);
    for (int r = 0; r <= G; ++r) zbs[size_t(r)] = uint32_t(uint64_t(sg.mg) * uint64_t(r) / uint64_t(G));
    if (zbs[size_t(rk)] != sg.zb || zbs[size_t(rk) + 1] != sg.zb + sg.nz)
        return fail(MVTV_BAD_ARG, "slab plane range differs from the even split of the communicator");
    const bool wd = P->wmode == W_DIAG;
    double w0 = 1.0, wstd = 0.0;   // mean and spread of W over the whole mesh
    {   // every rank must enqueue the same loop: the fused pass or not, the same edge layout (the z halo moves
        // whole planes in it), W or not. One sum of the flags, with the ranks' shares of sum W and sum W^2; a
        // mismatch fails on every rank alike
        // slot 7: this rank's block of every line can be cut into the line solves' segments (k_tris: <= 64
        // segments of <= 32 rows); checked here, before any rank enters a collective the infeasible one would skip
        const bool lines_ok = G == 1 || tri_slab_ok(sg.nz);
        double flags[9] = {P->f3d ? 1.0 : 0.0, P->g.eaos ? 1.0 : 0.0, P->e3d ? 1.0 : 0.0, double(sg.plane),
                           wd ? 1.0 : 0.0, P->wsum_own, P->wsum2_own, lines_ok ? 1.0 : 0.0, P->f4d ? 1.0 : 0.0};
        HIP_TRY(hipMemcpyAsync(P->red, flags, sizeof(flags), hipMemcpyHostToDevice, s));
        C->set_lane(0);
        MVTV_TRY(C->allreduce_sum(P->red, 9, s));
        double sum[9];
        HIP_TRY(hipMemcpyAsync(sum, P->red, sizeof(sum), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (int k = 0; k < 5; ++k)
            if (sum[k] != double(G) * flags[k]) return fail(MVTV_BAD_ARG, "slab ranks disagree on the loop layout");
        if (sum[8] != double(G) * flags[8]) return fail(MVTV_BAD_ARG, "slab ranks disagree on the loop layout");
        if (sum[7] != double(G))
            return fail(MVTV_BAD_ARG, "slab line solves: a rank's block of the last dimension has no split into <= 64 "
                                      "segments of <= 32 planes (e.g. a prime plane count above 64)");
        const double n_all = double(sg.plane) * double(sg.mg);
        if (wd) {
            w0 = sum[5] / n_all;
            wstd = std::sqrt(std::max(0.0, sum[6] / n_all - w0 * w0));
            if (!(w0 > 0.0)) w0 = 1.0;
        }
    }

    const double tol = opts->tol > 0 ? opts->tol : 1e-4;
    const int max_counter = opts->max_counter > 0 ? opts->max_counter : 3000;
    const bool fused = P->f3d;
    const bool fused4 = P->f4d;   // 4-D: edge update + the gather's pass A fused on the owned planes (k_admm4a)
    const bool pingpong = fused || fused4;
    // twin blocks (mvtv_internal.h twin_block): the run starts from u0 = 0, so the twins are equal whenever their
    // weights are (the same global deltas on every rank, hence the same choice); filled when the run ends
    // (4-D: the last owned plane's twins are filled before it goes to the next rank, whose ghost-plane pass A reads
    // every block of the halo)
    const bool twin = (fused || fused4) && twin_weights_equal(P->g, P->order) && !probe_env("MVTV_TWIN_OFF");
    if (P->timing && (fused || fused4)) P->twin_timed = twin;
    // folded right-hand side (as mvtv_capi.cpp's loop): the fused kernel stores s = rho (D^T alpha + D^T u) and the
    // next first pass reads oty + s (oty + (rho'/rho) s + rho' (c - 1) D^T u after a rho change)
    const uint32_t m0 = P->g.m[0];
    const bool fold_path = fused ? P->g.p == 3 : (P->g.p == 4 && P->e3d && P->g4 != nullptr && gather4_ok(P->g));
    const bool fold = fold_path && !wd && m0 >= 8 && m0 <= 4096 && (m0 & (m0 - 1)) == 0 &&
                      !probe_env("MVTV_FOLD_OFF") && !probe_env("MVTV_DCT_LDS");
    // interface buffers of the distributed line solves (16 numbers per line): the phase-1 numbers of this rank's
    // blocks by chunk (2 per line, the factorised form; 6 with the Thomas form of probe builds), the chunk's from
    // every rank, the 2 carries (Thomas: L, R values) by rank, and those of this rank's lines by chunk. One rank: the line solves are local, no buffers, no transfers,
    // unless MVTV_SLAB_DISTRIBUTED=1 asks for the distributed path at one rank (its transfers to itself),
    // which runs every collective call of the G-rank loop on one GPU
    const char* force = std::getenv("MVTV_SLAB_DISTRIBUTED");
    const bool solo = G == 1 && !(force && std::atoi(force) != 0);
    if (!solo && !P->slab_iface) MVTV_TRY(alloc(&P->slab_iface, 16 * size_t(sg.lines)));
    if (pingpong && !P->edges2) MVTV_TRY(alloc(&P->edges2, size_t(P->g.nb) * P->g.N));
    // the z ping-pong pair by timed probes, as one GPU's loop does (its first fused run, slabs of >= 2^24 nodes):
    // the fused pass's time depends on which physical buffers z moves between (slab world 1 at 512^3: 3.41 ms
    // on the allocation-order pair against 3.17 for the one-GPU loop in the same round-4 sweep); a rank-local
    // choice, no collective. Skipped where ranks share a device (more ranks than devices: the IPC rehearsals), whose
    // probes would time each other and race for the free memory the candidates need. The state is zeroed below
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    const bool shared_device = G > 1 && ndev > 0 && G > ndev;
    if (fused && !P->zpicked && !shared_device) MVTV_TRY(zpair_pick(P, false, twin));
    const size_t nodes = P->g.N, ebytes = size_t(P->g.nb) * nodes * sizeof(double);

    // ---- initial state: theta0 everywhere (ghosts included), u0 = 0, g_alpha = D^T D theta0 -----------
    HIP_TRY(launch_fill(s, P->theta, theta0, nodes));
    HIP_TRY(hipMemsetAsync(P->edges, 0, ebytes, s));
    if (pingpong) HIP_TRY(hipMemsetAsync(P->edges2, 0, ebytes, s));
    HIP_TRY(hipMemsetAsync(P->guprev, 0, nodes * sizeof(double), s));
    HIP_TRY(launch_apply_A(P->g, P->L(), 1.0, W_NONE, nullptr, P->theta, P->ga, nullptr, nullptr));
    AdmmCtl& c = *P->host_ctl;
    std::memset(&c, 0, sizeof(c));
    c.variant = MVTV_VARIANT_RCPP;
    c.fixed_iters = opts->fixed_iters > 0 ? opts->fixed_iters : 0;
    c.max_counter = max_counter;
    c.lambda = lambda;
    c.tol = tol;
    c.sqrtN = std::sqrt(double(P->g.N / P->g.m[p - 1]) * double(sg.mg));
    {   // global edge count: sum over blocks of prod_j (m_j - [j in S']) with the global last extent
        double E = 0.0;
        for (int k = 0; k < P->g.nb; ++k) {
            double len = 1.0;
            for (int j = 0; j < p; ++j) {
                const double mj = j == p - 1 ? double(sg.mg) : double(P->g.m[j]);
                len *= mj - double((P->sprime[k] >> j) & 1);
            }
            E += len;
        }
        c.sqrtE = std::sqrt(E);
    }
    c.rho = rho0;
    c.sigma = rho0;
    c.c_prev = 1.0;
    c.t_z = 0.0;
    c.t_next = lambda / rho0;
    c.counter = 1;
    c.dual_norm = c.primal_norm = 1.0;
    c.eps_dual = c.eps_pri = tol;
    HIP_TRY(hipMemcpyAsync(P->ctl, &c, sizeof(AdmmCtl), hipMemcpyHostToDevice, s));

    // geometry of the owned planes (local passes) and of this rank's line chunk (the last dimension)
    Geom og = P->g;
    og.m[p - 1] = sg.nz;
    og.N = sg.plane * sg.nz;
    og.ibeg = 0;
    og.iend = og.N;
    double* th = P->theta + sg.off;
    const size_t ln = sg.lines, ch = sg.chunk;
    double* co_send = P->slab_iface;          // [chunk s][6][line in chunk]
    double* co_recv = co_send + 6 * ln;       // [rank r][6][line in my chunk]
    double* lr_send = co_recv + 6 * ln;       // [rank r][2][line in my chunk]
    double* lr_recv = lr_send + 2 * ln;       // [chunk s][2][line in chunk]
    const double scale = 1.0 / double(sg.lines);   // the forward transforms along dims 0..p-2 (unnormalised)
    double* gbuf[2] = {P->guprev, P->gu};
    double* ebuf[2] = {P->edges, pingpong ? P->edges2 : P->edges};
    const size_t pl = sg.plane;
    const size_t first_owned = size_t(P->g_lo) * pl, last_owned = first_owned + size_t(sg.nz - 1) * pl;

    // The collectives run on their own stream sc, handed data by events, so the compute stream s goes on
    // (the z halo, needed by the next iteration's edge pass, runs during the next theta-solve). One rank: no
    // transfers, everything on s.
    hipStream_t sc = s;
    if (!solo) {
        if (!P->comm_stream) HIP_TRY(hipStreamCreateWithFlags(&P->comm_stream, hipStreamNonBlocking));
        sc = P->comm_stream;
    }
    struct Events {
        std::vector<hipEvent_t> v;
        ~Events() {
            for (auto e : v) (void)hipEventDestroy(e);
        }
    } evs;
    // coefficients ready / gathered, neighbour values ready / delivered, theta ready / halo done, sums ready /
    // reduced, edges ready / halo done, z halo done
    enum { EV_CO = 0, EV_COD, EV_LR, EV_LRD, EV_TH, EV_THD, EV_RED, EV_AR, EV_EDGE, EV_EDGED, EV_ZH, EV_N };
    for (int i = 0; i < EV_N; ++i) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.v.push_back(e);
    }
    hipEvent_t* ev = evs.v.data();
    auto handoff = [&](hipEvent_t e, hipStream_t from, hipStream_t to) -> mvtv_status {
        HIP_TRY(hipEventRecord(e, from));
        HIP_TRY(hipStreamWaitEvent(to, e, 0));
        return MVTV_OK;
    };
    bool zh_pending = false;   // a z halo was enqueued on sc that the next edge pass must wait for
    // Collectives on the critical path (the line solves' two all-to-alls, every all-reduce) go on the compute
    // stream itself, lane 0 of the transport, so no event hand-off between streams sits between a kernel and the
    // collective that consumes its output (a rank's share at G = 8 showed ~20 us of idle GPU per hand-off, eight per
    // iteration); the halos stay on sc, lane 1 (RCCL: a second communicator split off the first, so the two lanes may
    // run at once), the z halo overlapping the next theta-solve. One lane (lanes() == 1, or MVTV_SLAB_CRIT_SC=1 in
    // probe builds): every collective on sc with hand-offs, the round-4 schedule
    const bool crit_s = !solo && C->lanes() >= 2 && !probe_flag("MVTV_SLAB_CRIT_SC");
    auto lane = [&](int l) { C->set_lane(crit_s ? l : 0); };

    // edge plane e of buffer z (eaos: one contiguous run of nb * plane words; block-major: nb runs)
    auto edge_plane_xfer = [&](double* z, size_t e, int peer, bool is_send) -> mvtv_status {
        if (P->g.eaos) {
            double* ptr = z + e * pl * size_t(P->g.nb);
            return is_send ? C->send(ptr, pl * size_t(P->g.nb), peer, sc) : C->recv(ptr, pl * size_t(P->g.nb), peer, sc);
        }
        for (int k = 0; k < P->g.nb; ++k) {
            double* ptr = z + size_t(k) * nodes + e * pl;
            MVTV_TRY(is_send ? C->send(ptr, pl, peer, sc) : C->recv(ptr, pl, peer, sc));
        }
        return MVTV_OK;
    };
    // all-to-all of k numbers per line: block r of `send` (k x chunk) -> rank r, rank r's -> block r of `recv`
    auto a2a = [&](const double* send, double* recv, size_t k, hipStream_t st) -> mvtv_status {
        MVTV_TRY(C->begin());
        for (int r = 0; r < G; ++r) MVTV_TRY(C->send(send + size_t(r) * k * ch, k * ch, r, st));
        for (int r = 0; r < G; ++r) MVTV_TRY(C->recv(recv + size_t(r) * k * ch, k * ch, r, st));
        return C->end(st);
    };
    // a critical-path all-to-all / all-reduce: on s (lane 0), or on sc between hand-offs (one lane)
    auto crit_a2a = [&](const double* send, double* recv, size_t k, int e_in, int e_out) -> mvtv_status {
        lane(0);
        if (crit_s) return a2a(send, recv, k, s);
        MVTV_TRY(handoff(ev[e_in], s, sc));
        MVTV_TRY(a2a(send, recv, k, sc));
        return handoff(ev[e_out], sc, s);
    };
    auto crit_allreduce = [&](double* buf, size_t n) -> mvtv_status {
        lane(0);
        if (crit_s) return C->allreduce_sum(buf, n, s);
        MVTV_TRY(handoff(ev[EV_RED], s, sc));
        MVTV_TRY(C->allreduce_sum(buf, n, sc));
        return handoff(ev[EV_AR], sc, s);
    };

    // ghost planes of a node vector v (theta, or PCG's search direction): the first and last owned planes to
    // the neighbours, on sc, handed the data by event e and recording EV_THD when done
    auto halo = [&](double* v, hipEvent_t e) -> mvtv_status {
        MVTV_TRY(handoff(e, s, sc));
        lane(1);
        MVTV_TRY(C->begin());
        if (rk > 0) MVTV_TRY(C->send(v + first_owned, pl, rk - 1, sc));
        if (rk < G - 1) MVTV_TRY(C->send(v + last_owned, pl, rk + 1, sc));
        if (rk > 0) MVTV_TRY(C->recv(v, pl, rk - 1, sc));
        if (rk < G - 1) MVTV_TRY(C->recv(v + last_owned + pl, pl, rk + 1, sc));
        MVTV_TRY(C->end(sc));
        HIP_TRY(hipEventRecord(ev[EV_THD], sc));
        return MVTV_OK;
    };
    auto theta_halo = [&]() -> mvtv_status { return halo(P->theta, ev[EV_TH]); };

    // ---- W != I: the theta-solve (W + sigma D^T D) theta = b by PCG with the spectral preconditioner of
    //      A0 = mean(W) I + sigma D^T D (mvtv_capi.cpp pcgs_solve, the one-GPU solve), distributed: the
    //      operator on the owned planes after a halo of the search direction, the preconditioner as the direct
    //      slab solve (local passes + the substructured line solves), every dot product a local sum plus one
    //      all-reduce of 1-3 numbers, the PCG scalars on the device (identical on every rank, so every rank
    //      enqueues the same iterations and collectives). Host-synchronous per ADMM iteration: sigma, rho
    //      and the polls of the PCG come from the (identical) control block
    const double pcg_rtol = opts->pcg_rtol > 0 ? opts->pcg_rtol : 1e-10;
    const int pcg_maxit = opts->pcg_max_iter > 0 ? opts->pcg_max_iter : 20000;
    int pcg_total = 0, pcg_most = 0, pcg_unconv = 0, pcg_hint = 0;
    double cmean = 0.0;   // mean over the global mesh of D^T D's diagonal (pcgs_solve's dbar)
    for (int S = 1; S < (1 << p); ++S) {
        double prod = P->g.cS[S];
        for (int j = 0; j < p; ++j) {
            const double mj = j == p - 1 ? double(sg.mg) : double(P->g.m[j]);
            if ((S >> j) & 1) prod *= 2.0 * (mj - 1.0) / mj;
        }
        cmean += prod;
    }
    if (wd) {
        if (!P->p2) MVTV_TRY(alloc(&P->p2, nodes));
        if (!P->pcg_b) MVTV_TRY(alloc(&P->pcg_b, nodes));
        if (!P->pcg_s) MVTV_TRY(alloc(&P->pcg_s, nodes));
        if (!P->pcg_t) MVTV_TRY(alloc(&P->pcg_t, nodes));
    }
    // z = M0^-1 v on the owned planes (v and z offset to the first owned node)
    auto precond = [&](const double* v, double* z, double sigma, const int32_t* skip) -> mvtv_status {
        for (int d = 0; d <= p - 2; ++d)
            HIP_TRY(launch_dct_pass(P->spec, og, s, 0, d, d == 0 ? v : z, nullptr, 0.0, nullptr, 0.0, z, sigma, w0,
                                    nullptr, 0, 0.0, skip));
        if (solo) {
            HIP_TRY(launch_dct_pass(P->spec, og, s, 2, p - 1, z, nullptr, 0.0, nullptr, 0.0, z, sigma, w0, nullptr, 0,
                                    1.0 / (double(sg.lines) * double(sg.mg)), skip));
        } else {
            HIP_TRY(launch_tri_slab(P->spec, og, s, 1, z, co_send, nullptr, uint32_t(ch), rk > 0, rk < G - 1, scale,
                                    nullptr, sigma, w0, skip));
            MVTV_TRY(crit_a2a(co_send, co_recv, size_t(tri_slab_ncoef()), EV_CO, EV_COD));
            HIP_TRY(launch_tri_iface(P->spec, og, s, co_recv, lr_send, uint32_t(ch), G, rk, sg.mg, nullptr, sigma, w0,
                                     skip));
            MVTV_TRY(crit_a2a(lr_send, lr_recv, 2, EV_LR, EV_LRD));
            HIP_TRY(launch_tri_slab(P->spec, og, s, 3, z, nullptr, lr_recv, uint32_t(ch), rk > 0, rk < G - 1, scale,
                                    nullptr, sigma, w0, skip));
        }
        for (int d = p - 2; d >= 0; --d)
            HIP_TRY(launch_dct_pass(P->spec, og, s, 1, d, z, nullptr, 0.0, nullptr, 0.0, z, sigma, w0, nullptr, 0, 0.0,
                                    skip));
        return MVTV_OK;
    };
    // the global sum of nr per-workgroup partial rows, then k_finalize's PCG step `op` on it
    double* pred = P->red + 8;
    auto global_step = [&](int nparts, int nr, int op, double rtol2, int maxit) -> mvtv_status {
        HIP_TRY(launch_finalize(s, P->partials, nparts, nr, 0, 0, pred, P->st));
        if (!solo) MVTV_TRY(crit_allreduce(pred, size_t(nr)));
        HIP_TRY(launch_finalize(s, pred, 1, nr, 0, op, nullptr, P->st, rtol2, maxit));
        return MVTV_OK;
    };
    auto pcg_theta = [&](const double* gp) -> mvtv_status {
        const double sigma = c.sigma, rho = c.rho, cprev = c.c_prev;
        const Launch L{s, P->grid};
        Geom vg = og;   // the owned nodes as one vector
        const size_t off = sg.off;
        double *x = P->theta, *r = P->r, *z = P->q, *pv = P->p, *q = P->p2, *b = P->pcg_b;
        const double dbar = w0 + sigma * cmean;
        const bool scaled = wstd >= 0.1 * dbar;
        double* sinv = scaled ? P->pcg_s : nullptr;
        double* t = scaled ? P->pcg_t : nullptr;
        auto o = [&](double* v) { return v ? v + off : nullptr; };
        if (scaled) HIP_TRY(launch_pcgs_sinv(P->g, L, sigma, W_DIAG, P->wdiag, dbar, sinv));
        double* rin = scaled ? t : r;
        int h = P->tstart(MVTV_K_PCG_INIT);
        HIP_TRY(launch_apply_A(P->g, L, sigma, W_DIAG, P->wdiag, x, q, nullptr, nullptr));   // owned planes of A x
        P->tstop(h);
        HIP_TRY(launch_pcgs_vec(vg, L, 0, P->oty + off, P->ga + off, rho, gp + off, rho * cprev, x + off, r + off,
                                pv + off, q + off, nullptr, b + off, o(sinv), o(t), P->st, nullptr, 0));
        MVTV_TRY(precond(rin + off, z + off, sigma, nullptr));
        HIP_TRY(launch_pcgs_vec(vg, L, 2, nullptr, nullptr, 0.0, nullptr, 0.0, x + off, r + off, pv + off, q + off,
                                z + off, b + off, o(sinv), nullptr, P->st, P->partials, 1));
        MVTV_TRY(global_step(L.grid, PR_N, 1, pcg_rtol * pcg_rtol, pcg_maxit));
        HIP_TRY(hipMemcpyAsync(pv + off, z + off, size_t(og.N) * sizeof(double), hipMemcpyDeviceToDevice, s));
        const int32_t* skip = &P->st->done;
        auto iteration = [&]() -> mvtv_status {
            if (!solo) {   // the search direction's ghost planes
                MVTV_TRY(halo(pv, ev[EV_EDGE]));
                HIP_TRY(hipStreamWaitEvent(s, ev[EV_THD], 0));
            }
            int hh = P->tstart(MVTV_K_PCG_APPLY);
            HIP_TRY(launch_apply_A(P->g, L, sigma, W_DIAG, P->wdiag, pv, q, P->partials, P->st));   // q = A p, p.q
            P->tstop(hh);
            MVTV_TRY(global_step(L.grid, 1, 2, 0.0, 0));                                           // alpha
            HIP_TRY(launch_pcgs_vec(vg, L, 1, nullptr, nullptr, 0.0, nullptr, 0.0, x + off, r + off, pv + off, q + off,
                                    nullptr, b + off, o(sinv), o(t), P->st, nullptr, 0));
            MVTV_TRY(precond(rin + off, z + off, sigma, skip));                                   // z = M^-1 r
            HIP_TRY(launch_pcgs_vec(vg, L, 2, nullptr, nullptr, 0.0, nullptr, 0.0, x + off, r + off, pv + off, q + off,
                                    z + off, b + off, o(sinv), nullptr, P->st, P->partials, 0));
            MVTV_TRY(global_step(L.grid, PR_N, 3, 0.0, 0));                                        // beta, done
            HIP_TRY(launch_pcgs_vec(vg, L, 3, nullptr, nullptr, 0.0, nullptr, 0.0, x + off, r + off, pv + off, q + off,
                                    z + off, b + off, nullptr, nullptr, P->st, nullptr, 0));
            return MVTV_OK;
        };
        // polls as pcgs_solve: the last solve's count first, then every 2 iterations. The state is identical on
        // every rank, so every rank enqueues the same iterations
        int enq_pcg = 0, batch = pcg_hint > 0 ? std::max(2, pcg_hint) : kPcgPoll;
        for (;;) {
            for (int k = 0; k < batch && enq_pcg < pcg_maxit; ++k, ++enq_pcg) MVTV_TRY(iteration());
            HIP_TRY(hipMemcpyAsync(P->host_st, P->st, sizeof(PcgState), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (P->host_st->done || enq_pcg >= pcg_maxit) break;
            batch = 2;
        }
        const int pit = P->host_st->iter;
        pcg_hint = pit;
        pcg_total += pit;
        pcg_most = std::max(pcg_most, pit);
        const double relres = P->host_st->bnorm2 > 0 ? std::sqrt(P->host_st->rnorm2 / P->host_st->bnorm2) : 0.0;
        if (pit >= pcg_maxit && !(relres <= pcg_rtol)) {
            pcg_unconv += 1;
            if (opts->pcg_strict) return fail(MVTV_PCG_NOT_CONVERGED, "PCG hit pcg_max_iter");
        }
        if (!solo) {
            MVTV_TRY(theta_halo());
            HIP_TRY(hipStreamWaitEvent(s, ev[EV_THD], 0));
        }
        return MVTV_OK;
    };

    auto enqueue = [&](int j) -> mvtv_status {
        const int um = j == 0 ? U_EXPLICIT : U_FROM_Z;
        double* gp = gbuf[j & 1];
        double* gn = gbuf[(j + 1) & 1];
        double* zo = ebuf[j & 1];
        double* zn = ebuf[(j + 1) & 1];
        if (wd) {
            MVTV_TRY(pcg_theta(gp));
        } else {
            // -- theta-solve: forward passes along dims 0..p-2 on the owned planes, in place
            for (int d = 0; d <= p - 2; ++d) {
                const int h = P->tstart(d == 0 ? ((fold && j > 0) ? MVTV_K_DCT_FOLD : MVTV_K_DCT_FIRST) : MVTV_K_DCT);
                if (d == 0)
                    HIP_TRY(launch_dct_pass(P->spec, og, s, 0, 0, P->oty + sg.off, P->ga + sg.off, 0.0, gp + sg.off, 0.0,
                                            th, 0.0, 1.0, P->ctl, 0, 0.0, nullptr, nullptr, fold && j > 0));
                else
                    HIP_TRY(launch_dct_pass(P->spec, og, s, 0, d, th, nullptr, 0.0, nullptr, 0.0, th, 0.0, 1.0, P->ctl));
                P->tstop(h);
            }
            // -- the line solves along dim p-1
            if (solo) {   // the whole lines are here: the single-GPU pass (tridiagonal solve or DCT / divide / inverse)
                const int h = P->tstart(MVTV_K_DCT);
                HIP_TRY(launch_dct_pass(P->spec, og, s, 2, p - 1, th, nullptr, 0.0, nullptr, 0.0, th, 0.0, 1.0, P->ctl, 0,
                                        1.0 / (double(sg.lines) * double(sg.mg))));
                P->tstop(h);
            } else {
                int h = P->tstart(MVTV_K_DCT);
                HIP_TRY(launch_tri_slab(P->spec, og, s, 1, th, co_send, nullptr, uint32_t(ch), rk > 0, rk < G - 1, scale,
                                        P->ctl));
                P->tstop(h);
                MVTV_TRY(crit_a2a(co_send, co_recv, size_t(tri_slab_ncoef()), EV_CO, EV_COD));
                HIP_TRY(launch_tri_iface(P->spec, og, s, co_recv, lr_send, uint32_t(ch), G, rk, sg.mg, P->ctl));
                MVTV_TRY(crit_a2a(lr_send, lr_recv, 2, EV_LR, EV_LRD));
                h = P->tstart(MVTV_K_DCT);
                HIP_TRY(launch_tri_slab(P->spec, og, s, 3, th, nullptr, lr_recv, uint32_t(ch), rk > 0, rk < G - 1, scale,
                                        P->ctl));
                P->tstop(h);
            }
            // -- inverse passes along dims p-2..0, in place. The last one (dim 0) works plane by plane, so it
            //    transforms the first and last owned planes first and the halo carrying them overlaps the interior
            for (int d = p - 2; d >= 0; --d) {
                if (d == 0 && !solo && sg.nz >= 3) {
                    Geom one = og, mid = og;
                    one.m[p - 1] = 1;
                    one.N = sg.plane;
                    one.iend = one.N;
                    mid.m[p - 1] = sg.nz - 2;
                    mid.N = sg.plane * (sg.nz - 2);
                    mid.iend = mid.N;
                    double* edge_planes[2] = {th, th + size_t(sg.nz - 1) * pl};
                    for (double* ep : edge_planes) {
                        const int h = P->tstart(MVTV_K_DCT);
                        HIP_TRY(launch_dct_pass(P->spec, one, s, 1, 0, ep, nullptr, 0.0, nullptr, 0.0, ep, 0.0, 1.0, P->ctl));
                        P->tstop(h);
                    }
                    MVTV_TRY(theta_halo());
                    const int h = P->tstart(MVTV_K_DCT);
                    HIP_TRY(launch_dct_pass(P->spec, mid, s, 1, 0, th + pl, nullptr, 0.0, nullptr, 0.0, th + pl, 0.0, 1.0,
                                            P->ctl));
                    P->tstop(h);
                } else {
                    const int h = P->tstart(MVTV_K_DCT);
                    HIP_TRY(launch_dct_pass(P->spec, og, s, 1, d, th, nullptr, 0.0, nullptr, 0.0, th, 0.0, 1.0, P->ctl));
                    P->tstop(h);
                    if (d == 0 && !solo) MVTV_TRY(theta_halo());
                }
            }
            if (!solo) HIP_TRY(hipStreamWaitEvent(s, ev[EV_THD], 0));
        }
        // -- edge update + gather on the owned planes, partial sums into P->red
        if (fused) {
            if (zh_pending) HIP_TRY(hipStreamWaitEvent(s, ev[EV_ZH], 0));   // z_old's ghost plane is in place
            int h = P->tstart(MVTV_K_ADMM_FUSED);
            int npf = 0;
            HIP_TRY(launch_admm3d(P->g, P->order, um, s, P->theta, zo, zn, 0.0, 1.0, 0.0, 1.0, nullptr, P->ga, gn, gp,
                                  P->partials, &npf, P->ctl, fold, twin));
            P->tstop(h);
            HIP_TRY(launch_finalize(s, P->partials, npf, ER_N + GR_N, -(1 << ER_DTH), 0, P->red, P->st, 0.0, 0, P->ctl));
        } else if (fused4) {
            // z_new and pass A's sums of the owned planes in one pass; then the last owned plane of z_new to rank+1's
            // lower ghost plane, pass A on this rank's ghost plane (pass B at the first owned plane needs its Gw), pass B
            int h = P->tstart(MVTV_K_ADMM_FUSED4);
            int npe = 0;
            HIP_TRY(launch_admm4a(P->g, P->order, um, s, P->theta, zo, zn, 0.0, 1.0, 0.0, nullptr, P->g4, P->partials,
                                  &npe, P->ctl, twin));
            P->tstop(h);
            HIP_TRY(launch_finalize(s, P->partials, npe, ER_N, 1, 0, P->red, P->st, 0.0, 0, P->ctl));
            if (!solo && twin && rk < G - 1)
                HIP_TRY(fill_twins(P->g, P->order, s, zn, uint32_t(last_owned), uint32_t(last_owned + pl)));
            if (!solo) {
                MVTV_TRY(handoff(ev[EV_EDGE], s, sc));
                lane(1);
                MVTV_TRY(C->begin());
                if (rk < G - 1) MVTV_TRY(edge_plane_xfer(zn, last_owned / pl, rk + 1, true));
                if (rk > 0) MVTV_TRY(edge_plane_xfer(zn, 0, rk - 1, false));
                MVTV_TRY(C->end(sc));
                MVTV_TRY(handoff(ev[EV_EDGED], sc, s));
                if (rk > 0) HIP_TRY(launch_gather4a_ghost(P->g, P->order, s, zn, P->g4, P->ctl));
            }
            h = P->tstart(MVTV_K_GATHER4B);
            int npg = 0;
            HIP_TRY(launch_gather4b(P->g, U_FROM_Z, s, P->ga, gn, gp, 1.0, P->partials, &npg, P->ctl, P->g4, fold));
            P->tstop(h);
            HIP_TRY(launch_finalize(s, P->partials, npg, GR_N, 0, 0, P->red + ER_N, P->st, 0.0, 0, P->ctl));
        } else {
            int h = P->tstart(MVTV_K_EDGE_UPDATE);
            int npe = P->grid;
            if (P->e3d)
                HIP_TRY(launch_edge3d(P->g, P->order, um, s, P->theta, P->edges, 0.0, 1.0, 0.0, nullptr, P->partials,
                                      &npe, P->ctl));
            else
                HIP_TRY(launch_edge_update(P->g, P->order, um, P->L(), P->theta, P->edges, 0.0, 1.0, 0.0, nullptr,
                                           P->partials, P->ctl));
            P->tstop(h);
            HIP_TRY(launch_finalize(s, P->partials, npe, ER_N, 1, 0, P->red, P->st, 0.0, 0, P->ctl));
            // D^T at the first owned plane reads the new z of plane zb-1 (rank-1's last plane)
            if (!solo) {
                MVTV_TRY(handoff(ev[EV_EDGE], s, sc));
                lane(1);
                MVTV_TRY(C->begin());
                if (rk < G - 1) MVTV_TRY(edge_plane_xfer(P->edges, last_owned / pl, rk + 1, true));
                if (rk > 0) MVTV_TRY(edge_plane_xfer(P->edges, 0, rk - 1, false));
                MVTV_TRY(C->end(sc));
                MVTV_TRY(handoff(ev[EV_EDGED], sc, s));
            }
            h = P->tstart(MVTV_K_GATHER);
            const int hb = P->tstart_b(MVTV_K_GATHER4B);
            int npg = P->grid;
            if (P->e3d)
                HIP_TRY(launch_gather3d(P->g, P->order, U_FROM_Z, s, P->edges, 0.0, P->ga, gn, gp, 1.0, P->partials,
                                        &npg, P->ctl, P->g4, fold));
            else
                HIP_TRY(launch_gather(P->g, P->order, U_FROM_Z, P->L(), P->edges, 0.0, P->ga, gn, gp, 1.0,
                                      P->partials, P->ctl));
            P->tstop(h);
            P->tstop_b(hb);
            HIP_TRY(launch_finalize(s, P->partials, npg, GR_N, 0, 0, P->red + ER_N, P->st, 0.0, 0, P->ctl));
        }
        // -- global sums, then every rank's identical decision
        if (!solo) MVTV_TRY(crit_allreduce(P->red, ER_N + GR_N));
        HIP_TRY(launch_admm_control(s, P->ctl, P->red));
        // -- z halo for the next iteration's chunk-start recompute (fused): rank-1's last plane of z_new, on sc
        //    (z_new is complete: EV_RED was recorded after the fused pass) while s starts the next solve
        if (fused && !solo) {
            // z_new is complete on s (the fused pass and its sums precede this point); with the all-reduce on sc
            // its hand-off carried that, on s (crit_s) this one does
            if (crit_s) MVTV_TRY(handoff(ev[EV_EDGE], s, sc));
            lane(1);
            MVTV_TRY(C->begin());
            if (rk < G - 1) MVTV_TRY(edge_plane_xfer(zn, last_owned / pl, rk + 1, true));
            if (rk > 0) MVTV_TRY(edge_plane_xfer(zn, 0, rk - 1, false));
            MVTV_TRY(C->end(sc));
            HIP_TRY(hipEventRecord(ev[EV_ZH], sc));
            zh_pending = true;
        }
        return MVTV_OK;
    };

    // batches of iterations between polls: a schedule that depends only on the (identical) decisions, so
    // every rank enqueues the same collectives. Iterations enqueued past convergence are no-ops in their
    // kernels, but their collectives still move their buffers
    const int limit = opts->fixed_iters > 0 ? opts->fixed_iters : max_counter + 1;
    // (W != I: one iteration per poll, the PCG needs the control block's sigma on the host)
    // (tolerance mode: the last converged run's count first, as the one-GPU loop, so a warm-started path enqueues
    // few iterations past its stop; every rank holds the same hint)
    int target = wd ? 1 : (opts->fixed_iters > 0 ? opts->fixed_iters : (P->admm_hint > 0 ? P->admm_hint : 16));
    int enq = 0;
    std::vector<size_t> mark;
    for (;;) {
        while (enq < target && enq < limit) {
            mark.push_back(P->pending.size());
            MVTV_TRY(enqueue(enq++));
        }
        HIP_TRY(hipMemcpyAsync(P->host_ctl, P->ctl, sizeof(AdmmCtl), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (c.done || enq >= limit) break;
        target = wd ? enq + 1 : enq + std::max(4, enq / 4);
    }
    if (!solo) HIP_TRY(hipStreamSynchronize(sc));   // the last z halo
    const int it_done = c.it;
    if (P->timing && it_done < int(mark.size()))
        for (size_t e = mark[size_t(it_done)]; e < P->pending.size(); ++e) P->pending[e].kid = -1;
    P->harvest();
    if (P->timing && fold) P->fold_fix += c.nfix;
    if (opts->fixed_iters <= 0 && c.status == 0) P->admm_hint = it_done + 1;
    if (it_done & 1) {
        std::swap(P->guprev, P->gu);
        if (pingpong) std::swap(P->edges, P->edges2);
    }
    if (twin) {
        HIP_TRY(fill_twins(P->g, P->order, s, P->edges));
        HIP_TRY(hipStreamSynchronize(s));
    }
    P->twin_ok = true;
    P->edge_mode = it_done > 0 ? U_FROM_Z : U_EXPLICIT;
    P->t_z = c.t_z;
    P->c_state = c.c_prev;
    P->rho = c.rho;
    P->have_state = true;
    P->u_default = false;
    mvtv_admm_stats S{};
    S.iters = it_done;
    S.rho = c.rho;
    S.r_norm = c.r_norm;
    S.s_norm = c.s_norm;
    S.eps_pri = c.eps_pri;
    S.eps_dual = c.eps_dual;
    S.theta_solver = wd ? MVTV_SOLVER_PCG_SPECTRAL : MVTV_SOLVER_SPECTRAL;
    S.pcg_iters = pcg_total;
    S.pcg_iters_max = pcg_most;
    S.pcg_unconverged = pcg_unconv;
    S.status = c.status ? MVTV_MAXITER : MVTV_OK;
    S.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = S;
    return S.status == MVTV_OK ? MVTV_OK : MVTV_MAXITER;
}
}  // namespace

extern "C" mvtv_status mvtv_slab_run(mvtv_problem* P, mvtv_comm* C, const mvtv_admm_opts* opts, double lambda,
                                     double theta0, double rho0, mvtv_admm_stats* stats) {
    if (!C) return fail(MVTV_BAD_ARG, "null communicator");
    (void)C->run_begin();   // without a second lane on every rank (lanes() == 1) the loop keeps every collective on
                            // the collectives stream, the round-4 schedule; run_begin records no error
    const mvtv_status st =
        (!P || !opts) ? fail(MVTV_BAD_ARG, "null argument") : slab_run(P, C, opts, lambda, theta0, rho0, stats);
    if (st != MVTV_OK && st != MVTV_MAXITER) C->abort();
    return st;
}
