// rt_renderer.hip — render(scene, camera) -> frame in host memory on 1..N GPUs (host code).
//
// The reference renders one frame on one GPU and copies the float framebuffer to the host
// inside its timed region (G/src/main.cu:362-378; render() is G/include/query.h:13-29).  Here
// a frame is sharded over ranks as 8-row bands dealt round-robin (rank r renders bands
// b % world == r); each rank renders its bands into a contiguous device strip
// with the fused P6 epilogue (rt_render_device_p6).  The strips then reach the host frame by
// one of three paths, all with 2-D copies that put each band at its image rows (no un-permute
// pass):
//  * RCCL: one grouped ncclSend/ncclRecv per rank to rank 0's GPU (xGMI), then rank 0 copies
//    the assembled frame over its PCIe link (or keeps it in HBM, RT_DELIVER_DEVICE);
//  * DIRECT (one process driving every GPU): each GPU copies its own bands into the pinned
//    frame over its own PCIe link;
//  * HOST_SHARED (one process per GPU): the same per-rank copies into a host frame shared by
//    the processes (POSIX shared memory pinned in each), with per-rank completion words.
// Per rank three streams (compute, comm, copy) and per frame slot a strip buffer: frame k+1
// renders while frame k is gathered and copied to the host.
//
// RCCL is loaded at run time (dlopen "librccl.so.1"): in a process that has imported torch
// this is torch's own RCCL (same soname, already loaded), otherwise the image's.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>
#include <immintrin.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"
#include "rt_dma.hpp"

using rt::check_device;
using rt::DevBuf;
using rt::DeviceGuard;
using rt::hip_msg;
using rt::set_error;
using rt_dma::DmaCopier;
using rt_dma::Hsa;
using rt_dma::hsa;
using rt_dma::hsa_agents;
using rt_dma::hsa_now;

namespace {

// ---- RCCL, resolved at run time --------------------------------------------------------
struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            R.err = std::string("dlopen librccl.so.1: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp) {
                all = false;
                R.err += std::string(" missing ") + name;
            }
        };
        sym(R.GetUniqueId, "ncclGetUniqueId");
        sym(R.CommInitRank, "ncclCommInitRank");
        sym(R.CommInitAll, "ncclCommInitAll");
        sym(R.CommDestroy, "ncclCommDestroy");
        sym(R.GroupStart, "ncclGroupStart");
        sym(R.GroupEnd, "ncclGroupEnd");
        sym(R.Send, "ncclSend");
        sym(R.Recv, "ncclRecv");
        sym(R.GetErrorString, "ncclGetErrorString");
        R.ok = all;
    });
    return R;
}

int nccl_error(ncclResult_t e, const char* what) {
    const Rccl& R = rccl();
    return set_error(RT_ERR_COMM, std::string("RCCL ") + what + ": " +
                                      (R.GetErrorString ? R.GetErrorString(e) : std::to_string(int(e))));
}
#define NCCL_TRY(expr)                                    \
    do {                                                  \
        ncclResult_t e_ = (expr);                         \
        if (e_ != ncclSuccess) return nccl_error(e_, #expr); \
    } while (0)


constexpr int kTimeRing = 256;

// Bands of rank r (b % world == r) in its strip, in band order, go to image rows b*band_rows.
// The full bands are one strided 2-D copy; a partial last band (H % band_rows) a plain one.
// (The runtime moves these bytes with blit kernels, __amd_rocclr_copyBuffer, whatever
// GPU_BLIT_ENGINE_TYPE / HSA_ENABLE_SDMA say.  A 64-wave copy kernel of ours with 16-byte
// non-temporal stores into the pinned frame made the render kernel beside it far slower:
// 0.317 vs 0.251 ms per delivered c3 frame.)
hipError_t scatter_strip(char* dst, const char* strip, int r, int world, int H, int band_rows, size_t rb,
                         hipMemcpyKind kind, hipStream_t st) {
    if (world <= 1) return hipMemcpyAsync(dst, strip, size_t(H) * rb, kind, st);
    const int full = H / band_rows;  // bands 0 .. full-1 have band_rows rows
    const int nfull = full > r ? (full - 1 - r) / world + 1 : 0;
    const size_t band = size_t(band_rows) * rb;
    if (nfull > 0) {
        const hipError_t e = hipMemcpy2DAsync(dst + size_t(r) * band, size_t(world) * band, strip, band, band,
                                              size_t(nfull), kind, st);
        if (e != hipSuccess) return e;
    }
    if (H % band_rows != 0 && full % world == r) {  // band `full` is partial and ours
        const size_t rows = size_t(H - full * band_rows);
        return hipMemcpyAsync(dst + size_t(full) * band, strip + size_t(nfull) * band, rows * rb, kind, st);
    }
    return hipSuccess;
}

// ---- host frames shared by the processes of a job (RT_GATHER_HOST_SHARED) --------------
// One POSIX shared-memory segment per frame geometry: a header page of control words, then
// `depth` frame slots.  Rank 0's process creates it; every process maps it and pins the
// mapping with hipHostRegister, so each rank's device-to-host copy lands in the one frame.
// Control words (64-bit, one cache line each, accessed with __atomic builtins):
//   magic     written last by the creator: the header is complete
//   attached  local ranks of all processes that have pinned the segment (rank 0's process
//             unlinks the name once every rank has attached: nothing is left in /dev/shm)
//   released  frames [0, released) are no longer held by rank 0's caller (published at rank
//             0's submit of frame t: t - depth + 1); a rank copies frame t into its slot only
//             when released >= t - depth + 1
//   done[r]   frames [0, done[r]) of rank r are in the host frame (its copy finished)
constexpr uint64_t kShmMagic = 0x31564d4652544d52ull;  // "RMTRFMV1"
constexpr size_t kShmHeader = 8192;
constexpr size_t kOffMagic = 0, kOffGeom = 8, kOffAttached = 64, kOffReleased = 128, kOffDone = 192;
static_assert(kOffDone + 64 * 64 <= kShmHeader, "64 ranks of done words fit the header");

struct SharedFrames {
    std::string name;
    char* base = nullptr;
    size_t bytes = 0, slot_bytes = 0;
    bool registered = false, creator = false, unlinked = false;

    uint64_t* word(size_t off) const { return reinterpret_cast<uint64_t*>(base + off); }
    uint64_t* done(int r) const { return word(kOffDone + 64 * size_t(r)); }
    char* slot(int s) const { return base + kShmHeader + size_t(s) * slot_bytes; }
    static uint64_t load(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
    static void raise_to(uint64_t* p, uint64_t v) {  // monotone publish (one writer per word)
        if (__atomic_load_n(p, __ATOMIC_RELAXED) < v) __atomic_store_n(p, v, __ATOMIC_RELEASE);
    }
    void unlink_name() {
        if (creator && !unlinked && !name.empty()) (void)shm_unlink(name.c_str());
        unlinked = true;
    }
    void close() {
        if (registered) (void)hipHostUnregister(base);
        registered = false;
        if (base) (void)munmap(base, bytes);
        base = nullptr;
        unlink_name();
    }
    ~SharedFrames() { close(); }
};

double peer_timeout_s() {
    return std::max(0.1, rt::tuning(RT_TUNE_PEER_TIMEOUT_S, 120.0));
}

// Spin (then yield, then sleep) until pred() holds; false on timeout.
template <typename F>
bool spin_until(F pred) {
    if (pred()) return true;
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = peer_timeout_s();
    for (uint64_t i = 0;; ++i) {
        if (pred()) return true;
        if (i < 2000) {
#if !defined(__HIP_DEVICE_COMPILE__)
            __builtin_ia32_pause();
#endif
        } else if (i < 4000) {
            std::this_thread::yield();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(20));
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) return pred();
        }
    }
}

// Worker threads of an in-process renderer over several GPUs: a frame's host work per rank
// (the scene's pre-pass and render launches, the rank's copy) goes out in parallel, one thread
// per rank, so submitting a frame does not take N times one rank's host time.  run(n, job)
// runs job(0) on the caller and job(i) on worker i-1, and returns when all have finished; the
// first failing rank's code and message become the caller's.
class RankPool {
  public:
    ~RankPool() { stop(); }
    bool started() const { return !th_.empty(); }
    void start(int workers) {
        for (int i = 0; i < workers; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    void stop() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
        th_.clear();
        quit_ = false;
    }
    int run(int n, const std::function<int(int)>& job) {
        if (n <= 1 || th_.empty()) {
            for (int i = 0; i < n; ++i) {
                const int rc = job(i);
                if (rc != RT_OK) return rc;
            }
            return RT_OK;
        }
        rc_.assign(size_t(n), RT_OK);
        msg_.assign(size_t(n), std::string());
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &job;
            n_ = n;
            pending_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        rc_[0] = job(0);
        if (rc_[0] != RT_OK) msg_[0] = rt_last_error();
        {
            std::unique_lock<std::mutex> lk(m_);
            done_.wait(lk, [this] { return pending_ == 0; });
            job_ = nullptr;
        }
        for (int i = 0; i < n; ++i)
            if (rc_[i] != RT_OK) return set_error(rc_[i], msg_[i]);
        return RT_OK;
    }

  private:
    void loop(int w) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<int(int)>* job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            const int i = w + 1;
            if (job && i < n_) {
                rc_[i] = (*job)(i);
                if (rc_[i] != RT_OK) msg_[i] = rt_last_error();
            }
            {
                std::lock_guard<std::mutex> lk(m_);
                if (i < n_ && --pending_ == 0) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<int(int)>* job_ = nullptr;
    int n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
    std::vector<int> rc_;
    std::vector<std::string> msg_;
};

struct LocalRank {
    int device = 0;
    int rank = 0;  // global rank
    rt_scene* scene = nullptr;
    hipStream_t compute = nullptr, comm = nullptr, copy = nullptr;
    ncclComm_t nccl = nullptr;
    int rows = 0;                      // rows of this rank's strip for the current geometry
    std::vector<DevBuf> strip;         // per slot: rows*W*3 bytes (P6) or floats (F32)
    // Per slot.  The compute stream carries nothing but the scene's frame (its launches and its
    // own timing events): `rendered` is the scene's event after the frame's render kernel
    // (owned by the scene), nullptr when the rank has no rows.  `released` is what frees the
    // strip for reuse: released_ev (owned, recorded on comm/copy after the strip's last reader),
    // an alias of `rendered` (nothing reads the strip) or nullptr.
    std::vector<hipEvent_t> rendered, released, released_ev;
};

}  // namespace

struct rt_renderer {
    std::vector<LocalRank> ranks;
    int world = 1;
    int band_rows = 8;
    int deliver = RT_DELIVER_P6;
    int gather = RT_GATHER_DIRECT;
    int depth = 3;
    int flags = 0;
    bool rank0_local = false;  // ranks[0] is global rank 0
    // geometry the buffers are sized for
    int W = 0, H = 0, max_rows = 0;
    size_t row_bytes = 0, frame_bytes = 0, strip_cap = 0;
    // rank 0's side, per slot
    std::vector<DevBuf> gathered;       // RCCL: world strips of strip_cap bytes
    std::vector<DevBuf> dev_frame;      // RT_DELIVER_DEVICE
    std::vector<void*> host;            // host frames: pinned (hipHostMalloc) or slots of `shared`
    std::vector<hipEvent_t> delivered;  // per slot: delivered_ev[s], or rank 0's `rendered` (deliver none)
    std::vector<hipEvent_t> delivered_ev;  // owned, on ranks[0].copy
    std::vector<uint64_t> slot_ticket;  // frame held by each slot (+1; 0 = none)
    uint64_t next = 0;
    uint64_t first_valid = 0;           // tickets before the latest geometry change are gone
    // RT_GATHER_HOST_SHARED: the segment of the current geometry (every process)
    std::string shm_base;               // host_frame_name
    uint64_t shm_gen = 0;               // geometry generation (same sequence on every process)
    std::unique_ptr<SharedFrames> shared;
    // timing ring (rank 0's process): owned events on the comm / copy streams (gather start/end,
    // delivery start/end), and per frame and RT_TIME_* kind the (start, end) pair to read
    // (nullptr: the step did not run, 0 ms).  The frame's start is the scene's own first event.
    hipEvent_t tg0[kTimeRing] = {}, tg1[kTimeRing] = {}, td0[kTimeRing] = {}, td1[kTimeRing] = {};
    hipEvent_t ta[3][kTimeRing] = {}, tb[3][kTimeRing] = {};
    bool owns_scenes = true;
    RankPool pool;  // in-process renderers over several GPUs: per-rank submission threads
    // SDMA delivery (one rank, DIRECT, a host frame): per slot the copy's completion signal and
    // the HSA timestamp of the frame's submission; per ring entry the copy's and the frame's ms
    std::unique_ptr<DmaCopier> dma;
    std::vector<hsa_signal_t> dma_done;
    std::vector<uint64_t> dma_submit_ts;
    std::vector<bool> dma_pending;
    float dma_deliver_ms[kTimeRing] = {}, dma_frame_ms[kTimeRing] = {};
    bool dma_timed[kTimeRing] = {};

    ~rt_renderer() { release(); }
    // HOST_SHARED, after this process's copy streams were synchronised: publish every frame its
    // ranks copied, so rank 0 never waits on a frame whose "done" word only a wait would write
    // (a rank that resizes or closes without waiting its last tickets).
    void publish_copied() {
        if (!shared) return;
        uint64_t last = 0;
        for (uint64_t t : slot_ticket) last = std::max(last, t);
        if (last == 0) return;
        for (const LocalRank& L : ranks) SharedFrames::raise_to(shared->done(L.rank), last);
    }
    void release_buffers() {
        if (!shared) {
            for (void* h : host)
                if (h) (void)hipHostFree(h);
        }
        host.clear();
        shared.reset();
        gathered.clear();
        dev_frame.clear();
        for (LocalRank& L : ranks) {
            DeviceGuard g(L.device);
            L.strip.clear();
        }
    }
    void release() {
        pool.stop();
        if (dma) {  // every queued copy completes before its buffers go
            for (size_t i = 0; i < dma_done.size(); ++i)
                if (dma_pending[i]) (void)hsa().signal_wait(dma_done[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                                            HSA_WAIT_STATE_BLOCKED);
            dma.reset();
            for (hsa_signal_t d : dma_done) (void)hsa().signal_destroy(d);
            dma_done.clear();
        }
        for (LocalRank& L : ranks) {
            DeviceGuard g(L.device);
            if (L.compute) (void)hipStreamSynchronize(L.compute);
            if (L.comm) (void)hipStreamSynchronize(L.comm);
            if (L.copy) (void)hipStreamSynchronize(L.copy);
        }
        publish_copied();
        release_buffers();
        for (LocalRank& L : ranks) {
            DeviceGuard g(L.device);
            if (L.nccl && rccl().ok) (void)rccl().CommDestroy(L.nccl);
            L.nccl = nullptr;
            for (hipEvent_t e : L.released_ev) (void)hipEventDestroy(e);
            L.rendered.clear();
            L.released.clear();
            L.released_ev.clear();
            if (L.compute) (void)hipStreamDestroy(L.compute);
            if (L.comm) (void)hipStreamDestroy(L.comm);
            if (L.copy) (void)hipStreamDestroy(L.copy);
            L.compute = L.comm = L.copy = nullptr;
            if (owns_scenes && L.scene) rt_scene_destroy(L.scene);
            L.scene = nullptr;
        }
        if (!ranks.empty()) {
            DeviceGuard g(ranks[0].device);
            for (hipEvent_t e : delivered_ev) (void)hipEventDestroy(e);
            delivered.clear();
            delivered_ev.clear();
            for (hipEvent_t* ring : {tg0, tg1, td0, td1})
                for (int i = 0; i < kTimeRing; ++i)
                    if (ring[i]) (void)hipEventDestroy(ring[i]), ring[i] = nullptr;
        }
        ranks.clear();
    }
    bool uses_rccl() const { return gather == RT_GATHER_RCCL && deliver != RT_DELIVER_NONE; }
    bool host_shared() const { return gather == RT_GATHER_HOST_SHARED && deliver != RT_DELIVER_NONE; }
    size_t elem() const { return deliver == RT_DELIVER_F32 ? sizeof(float) : 1; }
};

extern "C" void rt_renderer_opts_default(rt_renderer_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->n_devices = 1;
    o->band_rows = 8;
    o->deliver = RT_DELIVER_P6;
    o->gather = RT_GATHER_AUTO;
    o->depth = 3;
}

extern "C" int rt_comm_unique_id(void* id128) {
    if (!id128) return set_error(RT_ERR_ARG, "rt_comm_unique_id: null");
    const Rccl& R = rccl();
    if (!R.ok) return set_error(RT_ERR_COMM, R.err);
    ncclUniqueId id;
    NCCL_TRY(R.GetUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id128, &id, sizeof(id));
    return RT_OK;
}

namespace {

int init_comms(rt_renderer* r, const rt_renderer_opts* o) {
    const Rccl& R = rccl();
    if (!R.ok) return set_error(RT_ERR_COMM, R.err);
    const int n = int(r->ranks.size());
    std::vector<ncclComm_t> comms(n, nullptr);
    if (r->world == n) {
        std::vector<int> devs(n);
        for (int i = 0; i < n; ++i) devs[i] = r->ranks[i].device;
        NCCL_TRY(R.CommInitAll(comms.data(), n, devs.data()));
    } else {
        ncclUniqueId id;
        std::memcpy(&id, o->unique_id, sizeof(id));
        NCCL_TRY(R.GroupStart());
        for (int i = 0; i < n; ++i) {
            HIP_TRY(hipSetDevice(r->ranks[i].device));
            const ncclResult_t e = R.CommInitRank(&comms[i], r->world, id, r->ranks[i].rank);
            if (e != ncclSuccess) {
                (void)R.GroupEnd();
                return nccl_error(e, "ncclCommInitRank");
            }
        }
        NCCL_TRY(R.GroupEnd());
    }
    for (int i = 0; i < n; ++i) r->ranks[i].nccl = comms[i];
    return RT_OK;
}

// Create (rank 0's process) or attach to (the others) the shared frames of the current
// geometry, pinned for device-to-host copies.
int open_shared(rt_renderer* r) {
    auto sf = std::make_unique<SharedFrames>();
    sf->name = r->shm_base + ".g" + std::to_string(r->shm_gen);
    sf->slot_bytes = (std::max<size_t>(r->frame_bytes, 1) + 4095) / 4096 * 4096;
    sf->bytes = kShmHeader + size_t(r->depth) * sf->slot_bytes;
    sf->creator = r->rank0_local;
    const uint64_t geom = (uint64_t(r->frame_bytes) << 16) ^ (uint64_t(r->depth) << 8) ^ uint64_t(r->world);
    if (sf->creator) {
        (void)shm_unlink(sf->name.c_str());  // a segment left by a crashed job of the same name
        const int fd = shm_open(sf->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) return set_error(RT_ERR_IO, "shm_open " + sf->name + ": " + std::strerror(errno));
        if (ftruncate(fd, off_t(sf->bytes)) != 0) {
            const int e = errno;
            ::close(fd);
            (void)shm_unlink(sf->name.c_str());
            return set_error(RT_ERR_NOMEM, "ftruncate " + sf->name + ": " + std::strerror(e));
        }
        // reserve the pages now: a tmpfs too small for the frames fails here with ENOSPC instead
        // of raising SIGBUS in whichever process first touches a missing page
        if (const int e = posix_fallocate(fd, 0, off_t(sf->bytes)); e != 0) {
            ::close(fd);
            (void)shm_unlink(sf->name.c_str());
            return set_error(RT_ERR_NOMEM, "posix_fallocate " + sf->name + " (" + std::to_string(sf->bytes) +
                                               " B in /dev/shm): " + std::strerror(e));
        }
        void* p = mmap(nullptr, sf->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (p == MAP_FAILED) {
            (void)shm_unlink(sf->name.c_str());
            return set_error(RT_ERR_NOMEM, "mmap " + sf->name + ": " + std::strerror(errno));
        }
        sf->base = static_cast<char*>(p);
        *sf->word(kOffGeom) = geom;
        __atomic_store_n(sf->word(kOffMagic), kShmMagic, __ATOMIC_RELEASE);
    } else {
        int err = 0;
        const bool ok = spin_until([&] {
            const int fd = shm_open(sf->name.c_str(), O_RDWR, 0600);
            if (fd < 0) return false;
            struct stat st;
            if (fstat(fd, &st) != 0 || size_t(st.st_size) < sf->bytes) {
                ::close(fd);
                return false;
            }
            void* p = mmap(nullptr, sf->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            ::close(fd);
            if (p == MAP_FAILED) {
                err = errno;
                return false;
            }
            char* b = static_cast<char*>(p);
            if (__atomic_load_n(reinterpret_cast<uint64_t*>(b + kOffMagic), __ATOMIC_ACQUIRE) != kShmMagic) {
                (void)munmap(p, sf->bytes);
                return false;
            }
            sf->base = b;
            return true;
        });
        if (!ok)
            return set_error(RT_ERR_COMM, "rank " + std::to_string(r->ranks[0].rank) + ": shared frame " + sf->name +
                                              " not created by rank 0's process" +
                                              (err ? std::string(" (mmap: ") + std::strerror(err) + ")" : ""));
        if (*sf->word(kOffGeom) != geom)
            return set_error(RT_ERR_ARG, "shared frame " + sf->name + ": processes disagree on frame size / depth / world");
    }
    HIP_TRY(hipHostRegister(sf->base, sf->bytes, hipHostRegisterPortable));
    sf->registered = true;
    __atomic_fetch_add(sf->word(kOffAttached), uint64_t(r->ranks.size()), __ATOMIC_ACQ_REL);
    r->host.assign(r->depth, nullptr);
    for (int s = 0; s < r->depth; ++s) r->host[s] = sf->slot(s);
    r->shared = std::move(sf);
    return RT_OK;
}

// Rank 0's process: remove the segment's name once every rank has pinned it.
void maybe_unlink(rt_renderer* r) {
    SharedFrames* sf = r->shared.get();
    if (sf && sf->creator && !sf->unlinked && SharedFrames::load(sf->word(kOffAttached)) >= uint64_t(r->world))
        sf->unlink_name();
}

// (Re)size every buffer for a W x H frame.  Waits for the frames in flight first; tickets
// submitted before the change can no longer be waited for.
int ensure_geometry(rt_renderer* r, int W, int H) {
    if (r->W == W && r->H == H && !r->ranks[0].strip.empty()) return RT_OK;
    for (LocalRank& L : r->ranks) {
        DeviceGuard g(L.device);
        HIP_TRY(hipStreamSynchronize(L.compute));
        HIP_TRY(hipStreamSynchronize(L.comm));
        HIP_TRY(hipStreamSynchronize(L.copy));
    }
    for (size_t i = 0; i < r->dma_pending.size(); ++i)  // SDMA copies still reading the buffers
        if (r->dma_pending[i]) {
            (void)hsa().signal_wait(r->dma_done[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            r->dma_pending[i] = false;
        }
    r->publish_copied();
    r->release_buffers();
    r->first_valid = r->next;
    r->W = W;
    r->H = H;
    r->row_bytes = size_t(W) * 3 * r->elem();
    r->frame_bytes = size_t(H) * r->row_bytes;
    r->max_rows = rt_shard_rows(H, r->band_rows, 0, r->world);  // rank 0 holds the most bands
    r->strip_cap = std::max<size_t>(size_t(r->max_rows) * r->row_bytes, 1);
    int rc;
    for (LocalRank& L : r->ranks) {
        DeviceGuard g(L.device);
        L.rows = rt_shard_rows(H, r->band_rows, L.rank, r->world);
        L.strip.resize(r->depth);
        for (DevBuf& b : L.strip)
            if ((rc = b.alloc(r->strip_cap)) != RT_OK) return rc;
        std::fill(L.rendered.begin(), L.rendered.end(), nullptr);
        std::fill(L.released.begin(), L.released.end(), nullptr);
    }
    std::fill(r->delivered.begin(), r->delivered.end(), nullptr);
    std::fill(r->slot_ticket.begin(), r->slot_ticket.end(), 0);
    if (r->host_shared()) {
        ++r->shm_gen;
        DeviceGuard g(r->ranks[0].device);
        if ((rc = open_shared(r)) != RT_OK) return rc;
    }
    if (r->rank0_local) {
        DeviceGuard g(r->ranks[0].device);
        if (r->uses_rccl()) {
            r->gathered.resize(r->depth);
            for (DevBuf& b : r->gathered)
                if ((rc = b.alloc(size_t(r->world) * r->strip_cap)) != RT_OK) return rc;
        }
        if (r->deliver == RT_DELIVER_DEVICE) {
            r->dev_frame.resize(r->depth);
            for (DevBuf& b : r->dev_frame)
                if ((rc = b.alloc(std::max<size_t>(r->frame_bytes, 1))) != RT_OK) return rc;
        } else if (r->deliver != RT_DELIVER_NONE && !r->host_shared()) {
            r->host.assign(r->depth, nullptr);
            for (void*& h : r->host)
                HIP_TRY(hipHostMalloc(&h, std::max<size_t>(r->frame_bytes, 1), hipHostMallocPortable));
        }
    }
    return RT_OK;
}

// HOST_SHARED: this process's ranks have frame `ticket` in the host frame (their copies are
// complete: the caller synchronised on them).
void publish_done(rt_renderer* r, uint64_t ticket) {
    if (!r->shared) return;
    for (const LocalRank& L : r->ranks) SharedFrames::raise_to(r->shared->done(L.rank), ticket + 1);
}

// SDMA delivery: wait for slot s's copy (of frame `ticket`) and keep its times.
int wait_dma(rt_renderer* r, int s, uint64_t ticket) {
    if (!r->dma || !r->dma_pending[s]) return RT_OK;
    const Hsa& H = hsa();
    (void)H.signal_wait(r->dma_done[s], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    r->dma_pending[s] = false;
    std::string msg;
    if (int rc = r->dma->error(&msg); rc != RT_OK) return set_error(rc, msg);
    hsa_amd_profiling_async_copy_time_t ct{};
    const int ring = int(ticket % kTimeRing);
    r->dma_timed[ring] = false;
    if (H.prof_copy_time(r->dma_done[s], &ct) == HSA_STATUS_SUCCESS && ct.end >= ct.start) {
        r->dma_deliver_ms[ring] = float(double(ct.end - ct.start) / double(H.ts_hz) * 1e3);
        r->dma_frame_ms[ring] = float(double(ct.end - std::min(ct.end, r->dma_submit_ts[s])) / double(H.ts_hz) * 1e3);
        r->dma_timed[ring] = true;
    }
    return RT_OK;
}

// Host wait until slot s may be reused (its previous frame fully delivered / released).
int wait_slot(rt_renderer* r, int s) {
    if (r->slot_ticket[s] == 0) return RT_OK;
    if (int rc = wait_dma(r, s, r->slot_ticket[s] - 1); rc != RT_OK) return rc;
    for (LocalRank& L : r->ranks) {
        DeviceGuard g(L.device);
        if (L.released[s]) HIP_TRY(hipEventSynchronize(L.released[s]));
    }
    if (r->rank0_local && r->delivered[s]) {
        DeviceGuard g(r->ranks[0].device);
        HIP_TRY(hipEventSynchronize(r->delivered[s]));
    }
    publish_done(r, r->slot_ticket[s] - 1);
    return RT_OK;
}

}  // namespace

extern "C" int rt_renderer_create(size_t P, const rt_bvh_node* nodes, const rt_aabb* aabbs, const rt_triangle* tris,
                                  const int32_t* objids, const rt_material* mats, int nmat, const rt_light* lights,
                                  int nlights, const rt_renderer_opts* o, rt_renderer** out) {
    if (!out) return set_error(RT_ERR_ARG, "rt_renderer_create: null out");
    *out = nullptr;
    rt_renderer_opts d;
    rt_renderer_opts_default(&d);
    if (!o) o = &d;
    const int n = o->n_devices;
    if (n < 1 || n > 64) return set_error(RT_ERR_ARG, "n_devices must be in 1..64");
    const int world = o->world_size > 0 ? o->world_size : n;
    if (world < n || world > 64 || o->rank0 < 0 || o->rank0 + n > world)
        return set_error(RT_ERR_ARG, "bad world_size / rank0 for n_devices (world_size <= 64)");
    if (o->band_rows < 1) return set_error(RT_ERR_ARG, "band_rows must be >= 1");
    if (o->deliver < RT_DELIVER_P6 || o->deliver > RT_DELIVER_NONE) return set_error(RT_ERR_ARG, "bad deliver");
    if (o->gather < RT_GATHER_AUTO || o->gather > RT_GATHER_HOST_SHARED) return set_error(RT_ERR_ARG, "bad gather");
    const int depth = o->depth == 0 ? 3 : o->depth;
    if (depth < 1 || depth > 8) return set_error(RT_ERR_ARG, "depth must be in 1..8");
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = o->devices ? o->devices[i] : i;
    const bool distinct = std::set<int>(devs.begin(), devs.end()).size() == size_t(n);
    const bool named = o->host_frame_name && o->host_frame_name[0];
    int gather = o->gather;
    if (gather == RT_GATHER_AUTO) {
        // every rank in this process: per-device copies (for RT_DELIVER_DEVICE, cross-device
        // 2-D copies into rank 0's HBM).  The RCCL gather over distinct GPUs is taken only when
        // asked for (RT_GATHER_RCCL): it has not yet run on a multi-GPU box, and an automatic
        // choice must not turn a configuration that works into an RT_ERR_COMM at create.
        if (world == n) gather = RT_GATHER_DIRECT;
        else gather = named ? RT_GATHER_HOST_SHARED : RT_GATHER_RCCL;
    }
    if ((o->flags & RT_RENDERER_SELF_SEND) && o->gather == RT_GATHER_AUTO) gather = RT_GATHER_RCCL;
    if (gather == RT_GATHER_DIRECT && world > n)
        return set_error(RT_ERR_UNSUPPORTED, "RT_GATHER_DIRECT needs every rank in this process");
    if (gather == RT_GATHER_RCCL && world > n && !o->unique_id)
        return set_error(RT_ERR_ARG, "RCCL across processes needs unique_id (rt_comm_unique_id on rank 0, shared with "
                                     "every process); or name a host_frame_name for RT_GATHER_HOST_SHARED");
    if (gather == RT_GATHER_RCCL && !distinct)
        return set_error(RT_ERR_UNSUPPORTED, "RCCL needs one rank per device; use RT_GATHER_DIRECT for repeated ids");
    if (gather == RT_GATHER_HOST_SHARED) {
        if (!named || o->host_frame_name[0] != '/' || std::strchr(o->host_frame_name + 1, '/') ||
            std::strlen(o->host_frame_name) > 200)
            return set_error(RT_ERR_ARG, "RT_GATHER_HOST_SHARED needs host_frame_name \"/name\" (no other '/')");
        if (o->deliver == RT_DELIVER_DEVICE)
            return set_error(RT_ERR_UNSUPPORTED, "RT_DELIVER_DEVICE needs RCCL (the frame is assembled on rank 0's GPU)");
    }
    for (int i = 0; i < n; ++i) {
        int rc = check_device(devs[i]);
        if (rc != RT_OK) return rc;
    }
    std::unique_ptr<rt_renderer> r(new (std::nothrow) rt_renderer());
    if (!r) return set_error(RT_ERR_NOMEM, "out of memory");
    r->world = world;
    r->band_rows = o->band_rows;
    r->deliver = o->deliver;
    r->gather = gather;
    r->depth = depth;
    r->flags = o->flags;
    r->rank0_local = o->rank0 == 0;
    if (named) r->shm_base = o->host_frame_name;
    r->ranks.resize(n);
    r->slot_ticket.assign(depth, 0);
    int rc;
    for (int i = 0; i < n; ++i) {
        LocalRank& L = r->ranks[i];
        L.device = devs[i];
        L.rank = o->rank0 + i;
        DeviceGuard g(L.device);
        // one host repack + upload, then device-to-device clones
        if (i == 0) rc = rt_scene_create(L.device, P, nodes, aabbs, tris, objids, mats, nmat, lights, nlights, &L.scene);
        else rc = rt_scene_clone(r->ranks[0].scene, L.device, &L.scene);
        if (rc != RT_OK) return rc;
        HIP_TRY(hipStreamCreateWithFlags(&L.compute, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&L.comm, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&L.copy, hipStreamNonBlocking));
        L.rendered.assign(depth, nullptr);
        L.released.assign(depth, nullptr);
        L.released_ev.assign(depth, nullptr);
        for (int s = 0; s < depth; ++s) HIP_TRY(hipEventCreateWithFlags(&L.released_ev[s], hipEventDisableTiming));
    }
    if (r->rank0_local) {
        DeviceGuard g(r->ranks[0].device);
        r->delivered.assign(depth, nullptr);
        r->delivered_ev.assign(depth, nullptr);
        for (int s = 0; s < depth; ++s) HIP_TRY(hipEventCreateWithFlags(&r->delivered_ev[s], hipEventDisableTiming));
        for (hipEvent_t* ring : {r->tg0, r->tg1, r->td0, r->td1})
            for (int i = 0; i < kTimeRing; ++i) HIP_TRY(hipEventCreate(&ring[i]));
    }
    if (r->uses_rccl() && (rc = init_comms(r.get(), o)) != RT_OK) return rc;
    // several GPUs in this process: one submission thread per further rank (RT_TUNE_RENDERER_THREADS
    // 0 submits every rank from the calling thread, for A/B; 1 uses the threads for repeated
    // device ids too, for tests on one GPU)
    const double threads = rt::tuning(RT_TUNE_RENDERER_THREADS, -1.0);
    const bool use_pool = threads < 0.0 ? distinct : threads != 0.0;
    if (n > 1 && use_pool) r->pool.start(n - 1);
    // RT_TUNE_COPY_ENGINE: -1 (default) SDMA where it applies, 0 the runtime's copies, 1 SDMA or
    // fail.  It applies to one rank delivering into a host frame over its own PCIe link.
    const double engine = rt::tuning(RT_TUNE_COPY_ENGINE, -1.0);
    const bool dma_fits = world == 1 && n == 1 && gather == RT_GATHER_DIRECT &&
                          (o->deliver == RT_DELIVER_P6 || o->deliver == RT_DELIVER_F32);
    if (engine != 0.0 && dma_fits) {
        hsa_agent_t ga{0}, ca{0};
        if (hsa_agents(r->ranks[0].device, &ga, &ca)) {
            r->dma_done.assign(depth, hsa_signal_t{0});
            for (hsa_signal_t& d : r->dma_done)
                if (hsa().signal_create(0, 0, nullptr, &d) != HSA_STATUS_SUCCESS)
                    return set_error(RT_ERR_HIP, "hsa_signal_create failed");
            r->dma_submit_ts.assign(depth, 0);
            r->dma_pending.assign(depth, false);
            const double cw = rt::tuning(RT_TUNE_COPY_WAIT, -1.0);
            r->dma = std::make_unique<DmaCopier>(ga, ca, cw == 1.0, cw >= 2.0 ? int(std::min(cw, 1000.0)) : 0);
        } else if (engine > 0.0) {
            return set_error(RT_ERR_UNSUPPORTED, "SDMA delivery unavailable: " + hsa().err);
        }
    } else if (engine > 0.0) {
        return set_error(RT_ERR_UNSUPPORTED, "SDMA delivery applies to one rank delivering into a host frame");
    }
    *out = r.release();
    return RT_OK;
}

extern "C" int rt_renderer_copy_engine(const rt_renderer* r) { return r && r->dma ? 1 : 0; }

extern "C" void rt_renderer_destroy(rt_renderer* r) { delete r; }

extern "C" rt_scene* rt_renderer_scene(rt_renderer* r, int i) {
    return (r && i >= 0 && i < int(r->ranks.size())) ? r->ranks[i].scene : nullptr;
}
extern "C" int rt_renderer_local_ranks(const rt_renderer* r) { return r ? int(r->ranks.size()) : 0; }

namespace {
// rt_renderer_submit (nf = 1) and rt_renderer_submit_pair (nf = 2: frames t and t+1 in two
// slots, one render launch per local rank, rt_render_device_pair).
int submit_frames(rt_renderer* r, const rt_camera* const* cams, int nf, const rt_render_opts* opts, uint64_t* ticket) {
    for (int f = 0; f < nf; ++f) {
        if (!r || !cams[f] || !opts) return set_error(RT_ERR_ARG, "rt_renderer_submit: null argument");
        if (cams[f]->pixel_width < 1 || cams[f]->pixel_height < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    }
    int rc = ensure_geometry(r, cams[0]->pixel_width, cams[0]->pixel_height);
    if (rc != RT_OK) return rc;
    const uint64_t t0 = r->next;
    uint64_t tk[2];
    int sl[2], rg[2];
    char* dsts[2] = {nullptr, nullptr};
    const bool f32 = r->deliver == RT_DELIVER_F32;
    const bool rccl_mode = r->uses_rccl();
    const bool self_send = rccl_mode && (r->flags & RT_RENDERER_SELF_SEND);
    const bool shared = r->host_shared();
    LocalRank& R0 = r->ranks[0];
    const hipMemcpyKind kind = r->deliver == RT_DELIVER_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    for (int f = 0; f < nf; ++f) {
        const uint64_t t = tk[f] = t0 + uint64_t(f);
        const int s = sl[f] = int(t % uint64_t(r->depth));
        // The slot's previous frame is waited for here, on the host: the streams below need no
        // waits for buffer reuse (every wait or event on the compute stream costs GPU time
        // between the frame's kernels).
        if ((rc = wait_slot(r, s)) != RT_OK) return rc;
        const int ring = rg[f] = int(t % kTimeRing);
        // HOST_SHARED: rank 0's caller gives up frame t - depth with this submit
        if (shared && r->rank0_local && t + 1 >= uint64_t(r->depth))
            SharedFrames::raise_to(r->shared->word(kOffReleased), t + 1 - uint64_t(r->depth));
        for (int k = 0; k < 3; ++k) r->ta[k][ring] = r->tb[k][ring] = nullptr;
        if (r->deliver != RT_DELIVER_NONE && (r->rank0_local || shared))
            dsts[f] = static_cast<char*>(r->deliver == RT_DELIVER_DEVICE ? r->dev_frame[s].p : r->host[s]);
        for (LocalRank& L : r->ranks) L.rendered[s] = L.released[s] = nullptr;
        if (r->rank0_local) r->delivered[s] = nullptr;
    }
    // 1. every local rank renders its bands into strip[s] (the scene's frames and nothing else
    // on its compute stream); DIRECT / HOST_SHARED: then copies its own bands into their rows of
    // the host frame over its own PCIe link (the same job, so with several GPUs in this process
    // each rank's host work runs on its own thread).
    const bool copies = !rccl_mode && r->deliver != RT_DELIVER_NONE;
    auto copy_job = [&](LocalRank& L, bool own, int f) -> int {
        const uint64_t t = tk[f];
        const int s = sl[f], ring = rg[f];
        char* dst = dsts[f];
        // With a frame shared by the job's processes, a rank other than 0's first waits for rank
        // 0's caller to give up this slot's previous frame (rank 0 publishes that at its submit).
        if (shared && !r->rank0_local && t + 1 >= uint64_t(r->depth) && L.rendered[s]) {
            const uint64_t need = t + 1 - uint64_t(r->depth);
            if (!spin_until([&] { return SharedFrames::load(r->shared->word(kOffReleased)) >= need; }))
                return set_error(RT_ERR_COMM, "rank " + std::to_string(L.rank) + ": rank 0 did not release frame " +
                                                  std::to_string(t - uint64_t(r->depth)) + " within the peer timeout (RT_TUNE_PEER_TIMEOUT_S)");
        }
        DeviceGuard g(L.device);
        if (own && r->dma && L.rendered[s]) {  // SDMA: queued by the copier once the frame is rendered
            hsa().signal_store(r->dma_done[s], 1);
            r->dma_submit_ts[s] = hsa_now();
            r->dma_pending[s] = true;
            r->dma->push({L.rendered[s], dst, L.strip[s].p, r->frame_bytes, r->dma_done[s]});
            return RT_OK;
        }
        if (own) {
            if (L.rendered[s]) HIP_TRY(hipStreamWaitEvent(L.copy, L.rendered[s], 0));
            HIP_TRY(hipEventRecord(r->td0[ring], L.copy));
        }
        if (!L.rendered[s]) return RT_OK;
        if (!own) HIP_TRY(hipStreamWaitEvent(L.copy, L.rendered[s], 0));
        HIP_TRY(scatter_strip(dst, static_cast<const char*>(L.strip[s].p), L.rank, r->world, r->H, r->band_rows,
                              r->row_bytes, kind, L.copy));
        if (!own) {
            HIP_TRY(hipEventRecord(L.released_ev[s], L.copy));
            L.released[s] = L.released_ev[s];
        }
        return RT_OK;
    };
    auto rank_job = [&](int i) -> int {
        LocalRank& L = r->ranks[i];
        const bool own = &L == &R0 && r->rank0_local;  // rank 0's copy: delivered_ev below
        if (L.rows > 0) {
            DeviceGuard g(L.device);
            rt_render_opts o = *opts;
            o.band_rows = r->band_rows;
            o.band_index = L.rank;
            o.band_count = r->world;
            void* buf[2] = {L.strip[sl[0]].p, L.strip[sl[nf - 1]].p};
            // the renderer waits for buffer reuse on the host: its own frames skip the scene's
            // wait for work queued before them on the compute stream (there is none but its
            // frames).  Only for this call: a borrowed view (rt_renderer_scene) stays stream-ordered.
            rt::scene_set_caller_ordered(L.scene, true);
            int q;
            if (nf == 2)
                q = rt_render_device_pair(L.scene, cams[0], cams[1], &o, f32 ? static_cast<float*>(buf[0]) : nullptr,
                                          f32 ? nullptr : static_cast<uint8_t*>(buf[0]),
                                          f32 ? static_cast<float*>(buf[1]) : nullptr,
                                          f32 ? nullptr : static_cast<uint8_t*>(buf[1]), L.compute);
            else
                q = rt_render_device_p6(L.scene, cams[0], &o, f32 ? static_cast<float*>(buf[0]) : nullptr, nullptr,
                                        nullptr, f32 ? nullptr : static_cast<uint8_t*>(buf[0]), L.compute);
            rt::scene_set_caller_ordered(L.scene, false);
            if (q != RT_OK) return q;
            for (int f = 0; f < nf; ++f) {
                hipEvent_t first = nullptr;
                rt::scene_frame_events(L.scene, &first, &L.rendered[sl[f]], nf - 1 - f);
                if (own) r->ta[RT_TIME_FRAME][rg[f]] = first;
            }
        }
        if (!copies) return RT_OK;
        for (int f = 0; f < nf; ++f)
            if (int q = copy_job(L, own, f); q != RT_OK) return q;
        return RT_OK;
    };
    if ((rc = r->pool.run(int(r->ranks.size()), rank_job)) != RT_OK) return rc;
    for (int f = 0; f < nf; ++f) r->slot_ticket[sl[f]] = tk[f] + 1;
    r->next = t0 + uint64_t(nf);
    if (ticket) *ticket = t0;
    // 2. per frame: the gather (RCCL) or the completion of the copies
    auto finish = [&](int f) -> int {
        const uint64_t t = tk[f];
        const int s = sl[f], ring = rg[f];
        char* dst = dsts[f];
        if (r->deliver == RT_DELIVER_NONE) {
            for (LocalRank& L : r->ranks) L.released[s] = L.rendered[s];
            if (r->rank0_local) r->delivered[s] = r->tb[RT_TIME_FRAME][ring] = R0.rendered[s];
            return RT_OK;
        }
        if (rccl_mode) {
            // 2. strips -> rank 0 (one group: every send and receive of this process)
            const Rccl& N = rccl();
            for (LocalRank& L : r->ranks) {
                DeviceGuard g(L.device);
                if (L.rendered[s]) HIP_TRY(hipStreamWaitEvent(L.comm, L.rendered[s], 0));
                if (&L == &R0 && r->rank0_local) HIP_TRY(hipEventRecord(r->tg0[ring], L.comm));
            }
            NCCL_TRY(N.GroupStart());
            for (LocalRank& L : r->ranks) {
                if (L.rank == 0 && !self_send) continue;
                const size_t bytes = size_t(L.rows) * r->row_bytes;
                if (bytes == 0) continue;
                const ncclResult_t e = N.Send(L.strip[s].p, bytes, ncclUint8, 0, L.nccl, L.comm);
                if (e != ncclSuccess) {
                    (void)N.GroupEnd();
                    return nccl_error(e, "ncclSend");
                }
            }
            if (r->rank0_local) {
                char* g0 = static_cast<char*>(r->gathered[s].p);
                for (int q = self_send ? 0 : 1; q < r->world; ++q) {
                    const size_t bytes = size_t(rt_shard_rows(r->H, r->band_rows, q, r->world)) * r->row_bytes;
                    if (bytes == 0) continue;
                    const ncclResult_t e = N.Recv(g0 + size_t(q) * r->strip_cap, bytes, ncclUint8, q, R0.nccl, R0.comm);
                    if (e != ncclSuccess) {
                        (void)N.GroupEnd();
                        return nccl_error(e, "ncclRecv");
                    }
                }
            }
            NCCL_TRY(N.GroupEnd());
            for (LocalRank& L : r->ranks) {
                if ((L.rank != 0 || self_send) && L.rows > 0) {  // the send was the strip's last reader
                    DeviceGuard g(L.device);
                    HIP_TRY(hipEventRecord(L.released_ev[s], L.comm));
                    L.released[s] = L.released_ev[s];
                }
            }
            // 3. rank 0: every strip to its image rows
            if (r->rank0_local) {
                DeviceGuard g(R0.device);
                HIP_TRY(hipEventRecord(r->tg1[ring], R0.comm));
                HIP_TRY(hipStreamWaitEvent(R0.copy, r->tg1[ring], 0));
                if (!self_send && R0.rendered[s]) HIP_TRY(hipStreamWaitEvent(R0.copy, R0.rendered[s], 0));
                HIP_TRY(hipEventRecord(r->td0[ring], R0.copy));
                const char* g0 = static_cast<const char*>(r->gathered[s].p);
                for (int q = 0; q < r->world; ++q) {
                    const char* src = (q == 0 && !self_send) ? static_cast<const char*>(R0.strip[s].p)
                                                             : g0 + size_t(q) * r->strip_cap;
                    HIP_TRY(scatter_strip(dst, src, q, r->world, r->H, r->band_rows, r->row_bytes, kind, R0.copy));
                }
                HIP_TRY(hipEventRecord(r->td1[ring], R0.copy));
                HIP_TRY(hipEventRecord(r->delivered_ev[s], R0.copy));
                r->delivered[s] = r->delivered_ev[s];
                if (!self_send && R0.rows > 0) R0.released[s] = r->delivered_ev[s];
                r->ta[RT_TIME_GATHER][ring] = r->tg0[ring];
                r->tb[RT_TIME_GATHER][ring] = r->tg1[ring];
                r->ta[RT_TIME_DELIVER][ring] = r->td0[ring];
                r->tb[RT_TIME_DELIVER][ring] = r->tb[RT_TIME_FRAME][ring] = r->td1[ring];
            }
            return RT_OK;
        }
        // 2'. DIRECT / HOST_SHARED: the copies went out with the ranks' jobs; rank 0's frame is
        // complete when every local copy is.
        if (r->dma && R0.rendered[s]) {  // SDMA: the strip is free and the frame delivered with the copy
            r->delivered[s] = nullptr;
            R0.released[s] = nullptr;
            r->ta[RT_TIME_DELIVER][ring] = r->tb[RT_TIME_DELIVER][ring] = r->tb[RT_TIME_FRAME][ring] = nullptr;
            r->dma_timed[ring] = false;
            return RT_OK;
        }
        if (r->rank0_local) {
            DeviceGuard g(R0.device);
            for (size_t i = 1; i < r->ranks.size(); ++i)  // the frame is complete when every local copy is
                if (r->ranks[i].released[s]) HIP_TRY(hipStreamWaitEvent(R0.copy, r->ranks[i].released[s], 0));
            HIP_TRY(hipEventRecord(r->td1[ring], R0.copy));
            HIP_TRY(hipEventRecord(r->delivered_ev[s], R0.copy));
            r->delivered[s] = r->delivered_ev[s];
            if (R0.rendered[s]) R0.released[s] = r->delivered_ev[s];
            r->ta[RT_TIME_DELIVER][ring] = r->td0[ring];
            r->tb[RT_TIME_DELIVER][ring] = r->tb[RT_TIME_FRAME][ring] = r->td1[ring];
        }
        if (shared) {
            maybe_unlink(r);
            // ranks with no rows have nothing to copy: their share of frame t is complete
            for (const LocalRank& L : r->ranks)
                if (!L.rendered[s]) SharedFrames::raise_to(r->shared->done(L.rank), t + 1);
        }
        return RT_OK;
    };
    for (int f = 0; f < nf; ++f)
        if ((rc = finish(f)) != RT_OK) return rc;
    return RT_OK;
}
}  // namespace

extern "C" int rt_renderer_submit(rt_renderer* r, const rt_camera* cam, const rt_render_opts* opts, uint64_t* ticket) {
    const rt_camera* cams[1] = {cam};
    return submit_frames(r, cams, 1, opts, ticket);
}

extern "C" int rt_renderer_submit_pair(rt_renderer* r, const rt_camera* cam_a, const rt_camera* cam_b,
                                       const rt_render_opts* opts, uint64_t* ticket_a) {
    if (!r || !cam_a || !cam_b || !opts) return set_error(RT_ERR_ARG, "rt_renderer_submit_pair: null argument");
    if (r->depth < 2) return set_error(RT_ERR_ARG, "rt_renderer_submit_pair: needs depth >= 2 (two frame slots)");
    // one frame size: else as two submits
    if (cam_a->pixel_width != cam_b->pixel_width || cam_a->pixel_height != cam_b->pixel_height) {
        uint64_t t = 0;
        int rc = rt_renderer_submit(r, cam_a, opts, &t);
        if (rc == RT_OK) rc = rt_renderer_submit(r, cam_b, opts, nullptr);
        if (ticket_a) *ticket_a = t;
        return rc;
    }
    const rt_camera* cams[2] = {cam_a, cam_b};
    return submit_frames(r, cams, 2, opts, ticket_a);
}

extern "C" int rt_renderer_wait(rt_renderer* r, uint64_t ticket, const void** frame, size_t* bytes) {
    if (frame) *frame = nullptr;
    if (bytes) *bytes = 0;
    if (!r) return set_error(RT_ERR_ARG, "rt_renderer_wait: null renderer");
    if (ticket >= r->next || ticket + uint64_t(r->depth) < r->next)
        return set_error(RT_ERR_ARG, "rt_renderer_wait: frame not submitted or no longer held");
    if (ticket < r->first_valid)
        return set_error(RT_ERR_ARG, "rt_renderer_wait: frame submitted before a change of the frame size");
    const int s = int(ticket % uint64_t(r->depth));
    if (int rc = wait_dma(r, s, ticket); rc != RT_OK) return rc;
    for (LocalRank& L : r->ranks) {
        DeviceGuard g(L.device);
        if (L.released[s]) HIP_TRY(hipEventSynchronize(L.released[s]));
        else if (L.rendered[s]) HIP_TRY(hipEventSynchronize(L.rendered[s]));
    }
    if (r->rank0_local) {
        DeviceGuard g(r->ranks[0].device);
        if (r->delivered[s]) HIP_TRY(hipEventSynchronize(r->delivered[s]));
    }
    if (r->host_shared()) {
        publish_done(r, ticket);
        maybe_unlink(r);
        if (r->rank0_local) {  // every rank's bands are in the frame
            for (int q = 0; q < r->world; ++q) {
                const uint64_t* w = r->shared->done(q);
                if (!spin_until([&] { return SharedFrames::load(w) >= ticket + 1; }))
                    return set_error(RT_ERR_COMM, "rank " + std::to_string(q) + " did not deliver frame " +
                                                      std::to_string(ticket) + " within the peer timeout (RT_TUNE_PEER_TIMEOUT_S)");
            }
        }
    }
    if (r->rank0_local) {
        if (r->deliver == RT_DELIVER_DEVICE) {
            if (frame) *frame = r->dev_frame[s].p;
            if (bytes) *bytes = r->frame_bytes;
        } else if (r->deliver != RT_DELIVER_NONE) {
            if (frame) *frame = r->host[s];
            if (bytes) *bytes = r->frame_bytes;
        }
    }
    return RT_OK;
}

extern "C" int rt_renderer_render(rt_renderer* r, const rt_camera* cam, const rt_render_opts* opts, void* out,
                                  size_t cap) {
    uint64_t t = 0;
    int rc = rt_renderer_submit(r, cam, opts, &t);
    if (rc != RT_OK) return rc;
    const void* f = nullptr;
    size_t n = 0;
    if ((rc = rt_renderer_wait(r, t, &f, &n)) != RT_OK) return rc;
    if (!r->rank0_local || r->deliver == RT_DELIVER_NONE) return RT_OK;
    if (!out || cap < n) return set_error(RT_ERR_ARG, "rt_renderer_render: output smaller than the frame");
    if (r->deliver == RT_DELIVER_DEVICE) {
        DeviceGuard g(r->ranks[0].device);
        HIP_TRY(hipMemcpy(out, f, n, hipMemcpyDeviceToHost));
    } else {
        std::memcpy(out, f, n);
    }
    return RT_OK;
}

extern "C" int rt_renderer_times(rt_renderer* r, int kind, float* ms_out, int max, int* n_out) {
    if (n_out) *n_out = 0;
    if (!r || max < 0 || (max > 0 && !ms_out) || kind < RT_TIME_GATHER || kind > RT_TIME_FRAME)
        return set_error(RT_ERR_ARG, "rt_renderer_times: bad args");
    if (!r->rank0_local) return RT_OK;
    DeviceGuard g(r->ranks[0].device);
    const uint64_t have = std::min<uint64_t>(r->next, uint64_t(kTimeRing));  // the ring keeps the last 256
    const int n = int(std::min<uint64_t>(have, uint64_t(max)));
    for (int k = 0; k < n; ++k) {
        const int i = int((r->next - uint64_t(n) + uint64_t(k)) % kTimeRing);
        hipEvent_t a = r->ta[kind][i], b = r->tb[kind][i];
        ms_out[k] = 0.0f;  // a step that did not run (no gather in DIRECT mode, no copy at deliver none)
        if (r->dma_timed[i] && kind != RT_TIME_GATHER) {  // SDMA: the copy's own timestamps (waited frames)
            ms_out[k] = kind == RT_TIME_DELIVER ? r->dma_deliver_ms[i] : r->dma_frame_ms[i];
            continue;
        }
        if (!a || !b) continue;
        HIP_TRY(hipEventSynchronize(b));
        HIP_TRY(hipEventElapsedTime(&ms_out[k], a, b));
    }
    if (n_out) *n_out = n;
    return RT_OK;
}

extern "C" int rt_render_reference_gpus(size_t P, int W, int H, const rt_camera* cam, rt_vec3 miss, int max_depth,
                                        int spp, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                                        const rt_triangle* tris, const int32_t* objids, const rt_material* mats,
                                        int nmat, const rt_light* lights, int nlights, int diffuse_bounce,
                                        int n_gpus, rt_vec3* output) {
    if (!cam || !output) return set_error(RT_ERR_ARG, "rt_render_reference_gpus: null argument");
    if (W != cam->pixel_width || H != cam->pixel_height)
        return set_error(RT_ERR_ARG, "W/H must match the camera's pixel dimensions");
    rt_renderer_opts ro;
    rt_renderer_opts_default(&ro);
    ro.n_devices = n_gpus;
    ro.deliver = RT_DELIVER_F32;
    ro.gather = n_gpus > 1 ? RT_GATHER_RCCL : RT_GATHER_DIRECT;  // float strips gathered to device 0
    ro.depth = 1;
    rt_renderer* r = nullptr;
    int rc = rt_renderer_create(P, nodes, aabbs, tris, objids, mats, nmat, lights, nlights, &ro, &r);
    if (rc != RT_OK) return rc;
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.max_depth = max_depth;
    o.spp = spp;
    o.diffuse_bounce = diffuse_bounce;
    o.miss_color = miss;
    rc = rt_renderer_render(r, cam, &o, output, size_t(W) * size_t(H) * sizeof(rt_vec3));
    rt_renderer_destroy(r);
    return rc;
}
