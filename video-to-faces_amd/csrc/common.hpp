// Shared runtime pieces of libvtf_hip.so: error state, HIP checks, a grow-only device
// arena per handle.  Compiled for gfx950 only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/vtf.h"

namespace vtf {

void set_error(const std::string& msg);

struct Error {
    int code;
    std::string msg;
};

#define VTF_HIP(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            throw ::vtf::Error{VTF_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
    } while (0)

#define VTF_CHECK(cond, code, msg)                                                         \
    do {                                                                                   \
        if (!(cond)) throw ::vtf::Error{(code), (msg)};                                    \
    } while (0)

// Catch-all wrapper for C entry points.
template <class F>
int guarded(F&& f) {
    try {
        f();
        return VTF_OK;
    } catch (const Error& e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return VTF_E_ARG;
    }
}

// Named grow-only device buffers: get(slot, bytes) returns a pointer valid until the next
// get() of the same slot with a larger size.  Sized for 288 GB HBM: no pooling games.
// Per-handle scratch slots that grow (x1.5) and never shrink.  An outgrown buffer is retired,
// not freed: hipFree synchronizes the whole device, which stalls every other stream (the
// concurrent lanes of the bench / a serving process) and would wait on kernels still queued
// on this buffer; retired buffers are released with the handle.
struct Arena {
    std::vector<void*> ptr;
    std::vector<size_t> cap;
    std::vector<void*> retired;
    // pinned host buffers mapped into the device address space ("mailboxes"): small tables the
    // host hands to a kernel and small results a kernel hands back are read / written there
    // directly, with no runtime blit copy (a pageable hipMemcpyAsync stages through a pinned
    // buffer and runs a copy kernel per call) -- the host reads results after a stream sync
    struct Mail {
        void* h;
        void* d;
    };
    std::vector<Mail> mptr;
    std::vector<size_t> mcap;
    std::vector<void*> mretired;
    ~Arena() {
        for (void* p : ptr)
            if (p) (void)hipFree(p);
        for (void* p : retired) (void)hipFree(p);
        for (const Mail& m : mptr)
            if (m.h) (void)hipHostFree(m.h);
        for (void* p : mretired) (void)hipHostFree(p);
    }
    // a mailbox of at least `bytes`; retired (not freed) when it grows, like get()
    Mail mail(int slot, size_t bytes) {
        if ((int)mptr.size() <= slot) {
            mptr.resize(slot + 1, Mail{nullptr, nullptr});
            mcap.resize(slot + 1, 0);
        }
        if (bytes == 0) bytes = 16;
        if (mcap[slot] < bytes) {
            if (mptr[slot].h) mretired.push_back(mptr[slot].h);
            const size_t b = ((bytes + bytes / 2) + 4095) & ~(size_t)4095;
            void* h = nullptr;
            void* d = nullptr;
            // coherent (fine-grained): the device reads and writes go to host memory uncached, so a
            // table rewritten by the host between launches is never read stale from the L2
            VTF_HIP(hipHostMalloc(&h, b, hipHostMallocMapped | hipHostMallocCoherent));
            VTF_HIP(hipHostGetDevicePointer(&d, h, 0));
            mptr[slot] = Mail{h, d};
            mcap[slot] = b;
        }
        return mptr[slot];
    }
    void* get(int slot, size_t bytes) {
        if ((int)ptr.size() <= slot) {
            ptr.resize(slot + 1, nullptr);
            cap.resize(slot + 1, 0);
        }
        if (bytes == 0) bytes = 16;
        if (cap[slot] < bytes) {
            if (ptr[slot]) retired.push_back(ptr[slot]);
            size_t b = bytes + bytes / 2;
            VTF_HIP(hipMalloc(&ptr[slot], b));
            cap[slot] = b;
        }
        return ptr[slot];
    }
    template <class T>
    T* get(int slot, size_t n) {
        return reinterpret_cast<T*>(get(slot, n * sizeof(T)));
    }
};

// Makes `device` the calling thread's current HIP device for the scope of one entry point
// (allocations and launches of a handle bound to cuda:1 must not land on cuda:0 when the
// caller's current device differs) and restores the caller's device afterwards.
struct DeviceGuard {
    int prev = -1, dev = -1;
    explicit DeviceGuard(int d) : dev(d) {
        if (d < 0) return;
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) VTF_HIP(hipSetDevice(d));
    }
    ~DeviceGuard() {
        if (dev >= 0 && prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};

// guarded() with the handle's device current for the call
template <class F>
int guarded_on(int device, F&& f) {
    return guarded([&] {
        DeviceGuard g(device);
        f();
    });
}

// Scratch of the stateless entry points (NMS, cosine dedupe / classify, blob): one arena per
// (device, stream), held under its own lock for the call.  A process-global arena would hand
// one device's buffer to a launch on another device, or one lane's buffer to a concurrent lane.
// A stream's scratch arena, locked for the caller: `keep` holds the slot alive (a concurrent
// vtf_release_stream only drops the registry's reference), `lock` serialises entry points on
// the stream.  Member order matters: the lock is released before the reference.
struct StreamScratch {
    std::shared_ptr<void> keep;
    Arena* ar;
    std::unique_lock<std::mutex> lock;
};
StreamScratch stream_scratch(hipStream_t st);
// the device a stream belongs to (the current device for the null stream)
int stream_device(hipStream_t st);

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Read-only weights through the constant address space: the compiler then emits scalar
// (s_load) loads for wave-uniform addresses even in kernels that also store to global memory.
#define VTF_CONST __attribute__((address_space(4)))
template <class T>
__device__ inline const VTF_CONST T* cptr(const T* p) {
    return (const VTF_CONST T*)p;
}

__host__ __device__ inline uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
// fp32 -> bf16 bits, round to nearest even (host-side weight packing)
inline uint16_t f2bf(float f) {
    uint32_t u = f2u(f);
    if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
    u += 0x7FFF + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}

// descending-order sort key of a float; every NaN maps to one key above +inf, as torch's sort
// treats NaNs as equal and greater than every number, and -0 maps to +0's key (torch compares
// them equal: a stable sort keeps them in index order, and the tie checks see them as a tie)
__host__ __device__ inline uint32_t desc_key(float f) {
    uint32_t u = f != f ? 0x7fc00000u : (f == 0.f ? 0u : f2u(f));
    uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ~asc;
}

}  // namespace vtf
