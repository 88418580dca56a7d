// Batched Dynamics plugin callables (include/pinoloco.h, pl_dyn_*).
//
// The reference's Dynamics classes return CasADi point functions (dynamics/*.py);
// drivers and retract code call them one point at a time.  Here one call evaluates
// a batch of points, one thread per point (k_dyn), on the handle's device; a handle
// created with device = -1 evaluates the same code on the host (used by the host
// side of the CasADi export and the CPU tests).  The math is dyn.h on top of the
// tree passes of rbd.h, i.e. the same code the OCP rows run.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/pinoloco.h"
#include "dyn.h"
#include "handles.h"
#include "rows.h"
#include "state.h"

struct pl_dyn {
  const pl_model* model;
  PlModel M;
  PlOcpConst O[2];   // contact frames: [0] feet only, [1] feet + external-force frame
  int device;
  hipStream_t stream;
  PlModel* dM;
  PlOcpConst* dO;
  double* buf;
  size_t cap;        // doubles in buf
};

__global__ __launch_bounds__(64) void k_dyn(const PlModel* M, const PlOcpConst* O, PlFrameRef F, int fn, int flags,
                                            int B, const double* in0, const double* in1, const double* in2,
                                            const double* in3, int l0, int l1, int l2, int l3, double* out, int lo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  pl::dyn_eval(*M, *O, F, fn, flags, in0 ? in0 + (size_t)b * l0 : nullptr, in1 ? in1 + (size_t)b * l1 : nullptr,
               in2 ? in2 + (size_t)b * l2 : nullptr, in3 ? in3 + (size_t)b * l3 : nullptr, out + (size_t)b * lo);
}

extern "C" int pl_dyn_create(const pl_model* model, const int* foot_frames, int ext_force_frame, int base_frame,
                             int device, pl_dyn** out) {
  if (!model || !foot_frames || !out) { pl_set_error("null argument"); return -1; }
  pl_dyn* d = new pl_dyn();
  d->model = model;
  d->M = model->m;
  for (int v = 0; v < 2; ++v) {
    PlOcpConst& O = d->O[v];
    memset(&O, 0, sizeof(O));
    O.nq = d->M.nq;
    O.nv = d->M.nv;
    O.nj = d->M.nq - 7;
    O.nfeet = 4;
    for (int k = 0; k < 4; ++k) {
      O.feet[k] = frame_ref(model, foot_frames[k]);
      if (!O.feet[k].valid) { pl_set_error("invalid foot frame %d", foot_frames[k]); delete d; return -1; }
    }
    O.ext = frame_ref(model, ext_force_frame);
    O.base = frame_ref(model, base_frame);
    O.nee = (v == 1 && O.ext.valid) ? 5 : 4;
    O.nf = 3 * O.nee;
  }
  d->device = device;
  d->stream = nullptr;
  d->dM = nullptr;
  d->dO = nullptr;
  d->buf = nullptr;
  d->cap = 0;
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      pl_set_error("hipSetDevice / hipStreamCreate(%d) failed", device);
      delete d;
      return -2;
    }
    if (hipMalloc(&d->dM, sizeof(PlModel)) != hipSuccess || hipMalloc(&d->dO, 2 * sizeof(PlOcpConst)) != hipSuccess ||
        hipMemcpy(d->dM, &d->M, sizeof(PlModel), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->dO, d->O, 2 * sizeof(PlOcpConst), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipGetLastError();
      pl_set_error("device upload of the dynamics tables failed");
      pl_dyn_destroy(d);
      return -2;
    }
  }
  *out = d;
  return 0;
}

extern "C" void pl_dyn_destroy(pl_dyn* d) {
  if (!d) return;
  if (d->device >= 0) {
    (void)hipSetDevice(d->device);
    if (d->stream) hipStreamSynchronize(d->stream);
    if (d->buf) hipFree(d->buf);
    if (d->dM) hipFree(d->dM);
    if (d->dO) hipFree(d->dO);
    if (d->stream) hipStreamDestroy(d->stream);
  }
  delete d;
}

extern "C" int pl_dyn_sizes(const pl_dyn* d, int fn, int flags, int* in_len, int* out_len) {
  if (!d || !in_len || !out_len) { pl_set_error("null argument"); return -1; }
  if (fn < 0 || fn >= PL_FN_COUNT) { pl_set_error("unknown dynamics function %d", fn); return -1; }
  if ((flags & 1) && !d->O[1].ext.valid) { pl_set_error("no external-force frame on this handle"); return -1; }
  pl::dyn_in_len(d->M, fn, d->O[flags & 1].nf, in_len);
  *out_len = pl::dyn_out_len(d->M, fn);
  return 0;
}

extern "C" int pl_dyn_eval(pl_dyn* d, int fn, int batch, int frame, int flags, const double* in0, const double* in1,
                           const double* in2, const double* in3, double* out) {
  if (!d || !out || batch < 0) { pl_set_error("bad arguments"); return -1; }
  if (fn < 0 || fn >= PL_FN_COUNT) { pl_set_error("unknown dynamics function %d", fn); return -1; }
  if ((flags & 1) && !d->O[1].ext.valid) { pl_set_error("no external-force frame on this handle"); return -1; }
  int len[4], lo = pl::dyn_out_len(d->M, fn);
  const PlOcpConst& O = d->O[flags & 1];
  pl::dyn_in_len(d->M, fn, O.nf, len);
  const double* in[4] = {in0, in1, in2, in3};
  for (int k = 0; k < 4; ++k)
    if (len[k] > 0 && !in[k]) { pl_set_error("input %d missing", k); return -1; }
  PlFrameRef F;
  memset(&F, 0, sizeof(F));
  const bool frame_fn = fn == PL_FN_FRAME_POS || fn == PL_FN_FRAME_VEL || fn == PL_FN_FRAME_JAC;
  if (frame_fn) {
    F = frame_ref(d->model, frame);
    if (!F.valid) { pl_set_error("invalid frame id %d", frame); return -1; }
    if (fn == PL_FN_FRAME_VEL && (flags & 2) && !O.base.valid) {
      pl_set_error("relative_to_base needs the base_link frame");
      return -1;
    }
  }
  if (batch == 0) return 0;
  if (d->device < 0) {  // host handle
    for (int b = 0; b < batch; ++b)
      pl::dyn_eval(d->M, O, F, fn, flags, len[0] ? in0 + (size_t)b * len[0] : nullptr,
                   len[1] ? in1 + (size_t)b * len[1] : nullptr, len[2] ? in2 + (size_t)b * len[2] : nullptr,
                   len[3] ? in3 + (size_t)b * len[3] : nullptr, out + (size_t)b * lo);
    return 0;
  }
  (void)hipSetDevice(d->device);
  (void)hipGetLastError();
  const size_t B = batch;
  const size_t need = B * ((size_t)len[0] + len[1] + len[2] + len[3] + lo);
  if (need > d->cap) {
    if (d->buf) hipFree(d->buf);
    d->buf = nullptr;
    d->cap = 0;
    PL_CHECK_HIP(hipMalloc(&d->buf, need * sizeof(double)));
    d->cap = need;
  }
  double* dptr[4];
  size_t off = 0;
  for (int k = 0; k < 4; ++k) {
    dptr[k] = len[k] ? d->buf + off : nullptr;
    if (len[k]) PL_CHECK_HIP(hipMemcpyAsync(dptr[k], in[k], B * len[k] * 8, hipMemcpyHostToDevice, d->stream));
    off += B * len[k];
  }
  double* dout = d->buf + off;
  hipLaunchKernelGGL(k_dyn, dim3((batch + 63) / 64), dim3(64), 0, d->stream, d->dM, d->dO + (flags & 1), F, fn, flags,
                     batch, dptr[0], dptr[1], dptr[2], dptr[3], len[0], len[1], len[2], len[3], dout, lo);
  PL_CHECK_HIP(hipGetLastError());
  PL_CHECK_HIP(hipMemcpyAsync(out, dout, B * lo * 8, hipMemcpyDeviceToHost, d->stream));
  PL_CHECK_HIP(hipStreamSynchronize(d->stream));
  return 0;
}
