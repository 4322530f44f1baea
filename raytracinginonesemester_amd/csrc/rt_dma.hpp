// rt_dma.hpp — SDMA (DMA engine) copies from device memory to pinned host memory through the
// HSA runtime, shared by the renderer's frame delivery (rt_renderer.hip) and the HW1 scene's
// (rt_hw1.hip).  Host code only.
#pragma once
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"

namespace rt_dma {

using rt::hip_msg;

// ---- SDMA copies through the HSA runtime ---------------------------------------------------
// The runtime's device-to-host copy (hipMemcpyAsync) runs as a blit kernel on the CUs beside the
// next frame's render kernel: a c3 frame's 6.2 MB P6 body takes ~0.125 ms of PCIe time, and the
// render kernel beside it lost ~10 us per frame (profiles/r05/exp/).  hsa_amd_memory_async_copy
// from device memory to system memory runs on a DMA (SDMA) engine instead.  It cannot wait for a
// HIP event on the device, so a copier thread waits for the frame's render event and queues the
// copy; its completion is an HSA signal the renderer waits for.  HSA is resolved at run time from
// the runtime HIP itself loaded (same soname: torch's in a torch process, else the image's).
struct Hsa {
    bool ok = false;
    std::string err;
    decltype(&hsa_init) init = nullptr;
    decltype(&hsa_iterate_agents) iterate_agents = nullptr;
    decltype(&hsa_agent_get_info) agent_get_info = nullptr;
    decltype(&hsa_signal_create) signal_create = nullptr;
    decltype(&hsa_signal_destroy) signal_destroy = nullptr;
    decltype(&hsa_signal_store_screlease) signal_store = nullptr;
    decltype(&hsa_signal_wait_scacquire) signal_wait = nullptr;
    decltype(&hsa_amd_memory_async_copy) async_copy = nullptr;
    decltype(&hsa_amd_profiling_async_copy_enable) prof_enable = nullptr;
    decltype(&hsa_amd_profiling_get_async_copy_time) prof_copy_time = nullptr;
    decltype(&hsa_system_get_info) system_get_info = nullptr;
    uint64_t ts_hz = 0;
};

inline const Hsa& hsa() {
    static Hsa H;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
        if (!h) h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            H.err = std::string("dlopen libhsa-runtime64.so.1: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp) {
                all = false;
                H.err += std::string(" missing ") + name;
            }
        };
        sym(H.init, "hsa_init");
        sym(H.iterate_agents, "hsa_iterate_agents");
        sym(H.agent_get_info, "hsa_agent_get_info");
        sym(H.signal_create, "hsa_signal_create");
        sym(H.signal_destroy, "hsa_signal_destroy");
        sym(H.signal_store, "hsa_signal_store_screlease");
        sym(H.signal_wait, "hsa_signal_wait_scacquire");
        sym(H.async_copy, "hsa_amd_memory_async_copy");
        sym(H.prof_enable, "hsa_amd_profiling_async_copy_enable");
        sym(H.prof_copy_time, "hsa_amd_profiling_get_async_copy_time");
        sym(H.system_get_info, "hsa_system_get_info");
        // (HIP initialised the runtime; hsa_init only counts one more user)
        if (all && H.init() != HSA_STATUS_SUCCESS) {
            all = false;
            H.err = "hsa_init failed";
        }
        if (all && (H.prof_enable(true) != HSA_STATUS_SUCCESS ||
                    H.system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &H.ts_hz) != HSA_STATUS_SUCCESS || !H.ts_hz)) {
            all = false;
            H.err = "HSA copy profiling unavailable";
        }
        H.ok = all;
    });
    return H;
}

inline uint64_t hsa_now() {
    uint64_t t = 0;
    (void)hsa().system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}

// The HSA GPU agent of HIP device `device` (by PCI domain / bus / device / function) and a CPU
// agent (the destination agent of a copy into system memory).
inline bool hsa_agents(int device, hsa_agent_t* gpu, hsa_agent_t* cpu) {
    const Hsa& H = hsa();
    if (!H.ok) return false;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return false;
    struct Q {
        const Hsa* H;
        uint32_t bdf, domain;
        hsa_agent_t gpu{0}, cpu{0};
        bool g = false, c = false;
    } q{&H, uint32_t(p.pciBusID) << 8 | uint32_t(p.pciDeviceID) << 3, uint32_t(p.pciDomainID)};
    auto cb = [](hsa_agent_t a, void* d) -> hsa_status_t {
        Q& q = *static_cast<Q*>(d);
        hsa_device_type_t t;
        if (q.H->agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !q.c) {
            q.cpu = a;
            q.c = true;
        } else if (t == HSA_DEVICE_TYPE_GPU) {
            uint32_t bdf = 0, dom = 0;
            (void)q.H->agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
            (void)q.H->agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
            if ((bdf & ~7u) == q.bdf && dom == q.domain) {
                q.gpu = a;
                q.g = true;
            }
        }
        return HSA_STATUS_SUCCESS;
    };
    if (H.iterate_agents(cb, &q) != HSA_STATUS_SUCCESS || !q.g || !q.c) return false;
    *gpu = q.gpu;
    *cpu = q.cpu;
    return true;
}

// One thread per renderer: for each queued frame, wait for its render event (spinning: the
// frames come every ~0.15 ms), then queue its SDMA copy, whose completion decrements `done`.
class DmaCopier {
  public:
    struct Job {
        hipEvent_t ready;
        void* dst;
        const void* src;
        size_t bytes;
        hsa_signal_t done;
    };
    // block: wait for a job's event with hipEventSynchronize (one runtime call per job) instead of
    // polling it with hipEventQuery (each poll takes the runtime's locks the submitting thread
    // needs for its launches; polling reacts sooner)
    // poll_us > 0: poll every poll_us microseconds (sleeping between polls) instead of spinning
    DmaCopier(hsa_agent_t gpu, hsa_agent_t cpu, bool block = false, int poll_us = 0)
        : gpu_(gpu), cpu_(cpu), block_(block), poll_us_(poll_us) {
        th_ = std::thread([this] { loop(); });
    }
    ~DmaCopier() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void push(const Job& j) {
        {
            std::lock_guard<std::mutex> lk(m_);
            q_.push_back(j);
        }
        cv_.notify_one();
    }
    // the first failure of the copier (its jobs' signals were completed so nobody hangs)
    int error(std::string* msg) {
        std::lock_guard<std::mutex> lk(m_);
        if (msg) *msg = err_;
        return rc_;
    }

  private:
    void loop() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [this] { return quit_ || !q_.empty(); });
                if (q_.empty()) return;  // quit_ with nothing left
                j = q_.front();
                q_.pop_front();
            }
            hipError_t e;
            if (block_) {
                e = hipEventSynchronize(j.ready);
            } else {
                for (uint32_t i = 0; (e = hipEventQuery(j.ready)) == hipErrorNotReady; ++i) {
                    if (poll_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(poll_us_));
                    else if (i < 4096) _mm_pause();
                    else std::this_thread::yield();
                }
            }
            const Hsa& H = hsa();
            hsa_status_t hs = HSA_STATUS_SUCCESS;
            if (e == hipSuccess) hs = H.async_copy(j.dst, cpu_, j.src, gpu_, j.bytes, 0, nullptr, j.done);
            if (e != hipSuccess || hs != HSA_STATUS_SUCCESS) {
                std::lock_guard<std::mutex> lk(m_);
                if (rc_ == RT_OK) {
                    rc_ = RT_ERR_HIP;
                    err_ = e != hipSuccess ? hip_msg(e, "render event (SDMA delivery)")
                                           : "hsa_amd_memory_async_copy failed: " + std::to_string(int(hs));
                }
                H.signal_store(j.done, 0);
            }
        }
    }
    hsa_agent_t gpu_, cpu_;
    bool block_ = false;
    int poll_us_ = 0;
    std::thread th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Job> q_;
    bool quit_ = false;
    int rc_ = RT_OK;
    std::string err_;
};

}  // namespace rt_dma
