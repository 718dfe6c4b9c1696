/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * CPU restatement of torchvision's NMS core (torchvision/csrc/ops/cpu/nms_kernel.cpp,
 * nms_kernel_impl), the third-party native op the reference calls at
 * src/videotofaces/detectors/mtcnn.py:196,205,219 and
 * src/videotofaces/detectors/operations/post.py:8 (via torchvision.ops.batched_nms).
 * torchvision is NOT installed in this image and is unpinned by the reference
 * (requirements.txt:1-10); this follows its published algorithm:
 *   areas = (x2 - x1) * (y2 - y1)                      (fp32 tensor ops, no fma)
 *   order = scores.sort(stable=true, descending=true)
 *   greedy: keep i if not suppressed; suppress j if inter/(area_i + area_j - inter) > thr
 *   with thr a C double, so the fp32 IoU is promoted to double for the compare.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no fma contraction, IEEE fp32).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float s; int64_t i; } si_t;

static int cmp_desc_stable(const void* a, const void* b) {
    const si_t* x = (const si_t*)a;
    const si_t* y = (const si_t*)b;
    /* torch's sort: NaN above every number, NaNs equal among themselves */
    const int xn = x->s != x->s, yn = y->s != y->s;
    if (xn != yn) return xn ? -1 : 1;
    if (x->s > y->s) return -1;
    if (x->s < y->s) return 1;
    return (x->i < y->i) ? -1 : (x->i > y->i);
}

/* boxes: [n,4] (x1,y1,x2,y2) fp32 row-major.  keep: out, up to n.  returns nkeep. */
int64_t ora_nms(const float* boxes, const float* scores, int64_t n, double thr, int64_t* keep) {
    if (n <= 0) return 0;
    float* areas = (float*)malloc(sizeof(float) * n);
    si_t* ord = (si_t*)malloc(sizeof(si_t) * n);
    uint8_t* sup = (uint8_t*)calloc(n, 1);
    for (int64_t i = 0; i < n; i++) {
        const float* b = boxes + 4 * i;
        volatile float w = b[2] - b[0];
        volatile float h = b[3] - b[1];
        areas[i] = w * h;
        ord[i].s = scores[i];
        ord[i].i = i;
    }
    qsort(ord, n, sizeof(si_t), cmp_desc_stable);
    int64_t nk = 0;
    for (int64_t _i = 0; _i < n; _i++) {
        int64_t i = ord[_i].i;
        if (sup[i]) continue;
        keep[nk++] = i;
        const float* bi = boxes + 4 * i;
        float ix1 = bi[0], iy1 = bi[1], ix2 = bi[2], iy2 = bi[3], iarea = areas[i];
        for (int64_t _j = _i + 1; _j < n; _j++) {
            int64_t j = ord[_j].i;
            if (sup[j]) continue;
            const float* bj = boxes + 4 * j;
            float xx1 = ix1 > bj[0] ? ix1 : bj[0];
            float yy1 = iy1 > bj[1] ? iy1 : bj[1];
            float xx2 = ix2 < bj[2] ? ix2 : bj[2];
            float yy2 = iy2 < bj[3] ? iy2 : bj[3];
            float w = xx2 - xx1; if (w < 0.f) w = 0.f;
            float h = yy2 - yy1; if (h < 0.f) h = 0.f;
            volatile float inter = w * h;
            volatile float den = (iarea + areas[j]) - inter;
            float ovr = inter / den;
            if ((double)ovr > thr) sup[j] = 1;
        }
    }
    free(areas); free(ord); free(sup);
    return nk;
}
