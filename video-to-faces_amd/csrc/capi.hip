// C-ABI glue: error state, version, standalone box ops (include/vtf.h).
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "common.hpp"
#include "nms.hpp"

namespace vtf {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

__global__ void k_i64_to_i32(const int64_t* in, int64_t n, int32_t* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (int32_t)in[i];
}
__global__ void k_i32_to_i64(const int32_t* in, int64_t n, int64_t* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (int64_t)in[i];
}

int stream_device(hipStream_t st) {
    int dev = 0;
    if (st) {
        VTF_HIP(hipStreamGetDevice(st, &dev));
    } else {
        VTF_HIP(hipGetDevice(&dev));
    }
    return dev;
}

namespace {
struct Slot {
    std::mutex mu;
    Arena ar;
};
std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, std::shared_ptr<Slot>> g_slots;
}  // namespace

StreamScratch stream_scratch(hipStream_t st) {
    const int dev = stream_device(st);
    std::shared_ptr<Slot> s;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& p = g_slots[{dev, st}];
        if (!p) p = std::make_shared<Slot>();
        s = p;  // a reference taken under g_mu: a concurrent release cannot free the slot under us
    }
    Arena* ar = &s->ar;
    std::unique_lock<std::mutex> lk(s->mu);
    return StreamScratch{std::move(s), ar, std::move(lk)};
}

void release_dma_ws(hipStream_t st);

}  // namespace vtf

using namespace vtf;

extern "C" {

const char* vtf_last_error(void) { return g_err.c_str(); }

int vtf_version(void) { return 1; }

// The caller must not enqueue work on the stream from another thread during the release: the
// slot's arena is freed once the last entry point that already holds it returns (its
// StreamScratch keeps a reference), after this call has dropped the registry's.
int vtf_release_stream(void* hip_stream) {
    hipStream_t st = (hipStream_t)hip_stream;
    return guarded_on(stream_device(st), [&] {
        VTF_HIP(hipStreamSynchronize(st));
        std::shared_ptr<Slot> s;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            auto it = g_slots.find({stream_device(st), st});
            if (it != g_slots.end()) {
                s = std::move(it->second);
                g_slots.erase(it);
            }
        }
        if (s) {
            std::lock_guard<std::mutex> lk(s->mu);  // wait for an entry point still inside
        }
        s.reset();  // freed here, or by the last StreamScratch still holding it
        release_dma_ws(st);
    });
}

int vtf_batched_nms(const float* d_boxes, const float* d_scores, const int64_t* d_idxs, int64_t n,
                    double iou_threshold, int64_t* d_keep, int64_t* out_nkeep, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(out_nkeep && n >= 0, VTF_E_ARG, "bad argument");
        *out_nkeep = 0;
        if (n == 0) return;
        VTF_CHECK(d_boxes && d_scores && d_idxs && d_keep, VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        StreamScratch sc = stream_scratch(st);
        Arena& ar = *sc.ar;
        int32_t* img = ar.get<int32_t>(0, n);
        int32_t* call = ar.get<int32_t>(1, n);
        int32_t* keep = ar.get<int32_t>(2, n);
        k_i64_to_i32<<<cdiv(n, 256), 256, 0, st>>>(d_idxs, n, img);
        VTF_HIP(hipMemsetAsync(call, 0, n * 4, st));
        // the vanilla segment count is max id + 1.  Above torchvision's coordinate-trick bound
        // (n * 4 > 4000: one NMS per distinct id, results merged by score) the id values only
        // group the boxes, so they are remapped to their ranks among the distinct ids (any
        // category id works, as in torchvision); the trick path keeps them: its offsets are
        // idx * (max coordinate + 1), so the values set the fp32 rounding
        int32_t mx = 0;
        std::vector<int32_t> h(n);
        VTF_HIP(hipMemcpyAsync(h.data(), img, n * 4, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        for (int32_t v : h) {
            VTF_CHECK(v >= 0, VTF_E_ARG, "batched_nms: negative class ids are not supported");
            mx = v > mx ? v : mx;
        }
        if (n * 4 > 4000 && mx >= 1) {
            std::vector<int32_t> u(h);
            std::sort(u.begin(), u.end());
            u.erase(std::unique(u.begin(), u.end()), u.end());
            if ((int64_t)u.size() < (int64_t)mx + 1) {
                for (auto& v : h) v = (int32_t)(std::lower_bound(u.begin(), u.end(), v) - u.begin());
                mx = (int32_t)u.size() - 1;
                VTF_HIP(hipMemcpyAsync(img, h.data(), n * 4, hipMemcpyHostToDevice, st));
            }
        }
        std::vector<int64_t> nk;
        nms_multi(ar, d_boxes, d_scores, img, call, {n}, mx + 1, iou_threshold, keep, nk, st);
        k_i32_to_i64<<<cdiv(nk[0] > 0 ? nk[0] : 1, 256), 256, 0, st>>>(keep, nk[0], d_keep);
        VTF_HIP(hipStreamSynchronize(st));
        *out_nkeep = nk[0];
    });
}

}  // extern "C"
