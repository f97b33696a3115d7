// TORCH_LIBRARY(fsmi): the hot-path entry points of libfsmi.so (include/fsmi.h) registered as
// PyTorch operators, so a caller can reach them as torch.ops.fsmi.<name> (TorchScript, torch.library,
// the dispatcher) instead of the ctypes front end in ops.py.  Plain C++ (no device code): every op
// checks its tensors, allocates outputs through the caching allocator, and calls the C ABI on the
// current HIP stream of the input's device.  Built in-tree by torch.utils.cpp_extension
// (foundationstereo_amd/torch_ops.py) and linked against libfsmi.so.
//
// Reference interfaces these ops stand in for:
//   gwc_volume          core/submodule.py:399-412      concat_volume     core/submodule.py:416-427
//   allpairs_corr       core/geometry.py:24-40,68-77   volume_pyramid    core/geometry.py:29,34-36
//   geo_lookup          core/geometry.py:43-65         bilinear_sampler  core/utils/utils.py:44-55
//   disparity_regression core/submodule.py:431-435     softmax_regression core/foundation_stereo.py:218-220
//   context_upsample    core/submodule.py:456-468      softmax_context_upsample core/foundation_stereo.py:187-189
#include <torch/library.h>
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "../../include/fsmi.h"

namespace {

using at::Tensor;

void check_dev(const char* name, const Tensor& t) {
  TORCH_CHECK(t.is_cuda(), name, ": fsmi ops run on ROCm (HIP) device tensors only; got ", t.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, ": expected float32, got ", t.scalar_type());
}

// contiguous and 16-byte aligned: the kernels issue float4 accesses
Tensor dense(const Tensor& t) {
  Tensor c = t.contiguous();
  if (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 != 0) c = c.clone();
  return c;
}

void* stream_of(const Tensor& t) {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream(t.get_device()).stream());
}

void ok(int rc, const char* name) {
  TORCH_CHECK(rc == 0, "fsmi ", name, " failed (", rc, "): ", fsmi_last_error());
}

const float* cp(const Tensor& t) { return t.data_ptr<float>(); }
float* mp(Tensor& t) { return t.data_ptr<float>(); }

Tensor gwc_volume(const Tensor& fl_, const Tensor& fr_, int64_t maxdisp, int64_t num_groups) {
  const c10::DeviceGuard guard(fl_.device());   // launch + allocate on the tensors' device
  check_dev("gwc_volume", fl_); check_dev("gwc_volume", fr_);
  TORCH_CHECK(fl_.dim() == 4 && fl_.sizes() == fr_.sizes(), "gwc_volume: fl, fr must be (B,C,H,W) alike");
  Tensor fl = dense(fl_), fr = dense(fr_);
  const int64_t B = fl.size(0), C = fl.size(1), H = fl.size(2), W = fl.size(3);
  Tensor out = at::empty({B, num_groups, maxdisp, H, W}, fl.options());
  ok(fsmi_gwc_volume(cp(fl), cp(fr), mp(out), B, C, num_groups, maxdisp, H, W, stream_of(fl)), "gwc_volume");
  return out;
}

Tensor concat_volume(const Tensor& pl_, const Tensor& pr_, int64_t maxdisp) {
  const c10::DeviceGuard guard(pl_.device());
  check_dev("concat_volume", pl_); check_dev("concat_volume", pr_);
  TORCH_CHECK(pl_.dim() == 4 && pl_.sizes() == pr_.sizes(), "concat_volume: pl, pr must be (B,C,H,W) alike");
  Tensor pl = dense(pl_), pr = dense(pr_);
  const int64_t B = pl.size(0), C = pl.size(1), H = pl.size(2), W = pl.size(3);
  Tensor out = at::empty({B, 2 * C, maxdisp, H, W}, pl.options());
  ok(fsmi_concat_volume(cp(pl), cp(pr), mp(out), B, C, maxdisp, H, W, stream_of(pl)), "concat_volume");
  return out;
}

std::vector<Tensor> allpairs_corr(const Tensor& fl_, const Tensor& fr_, int64_t num_levels) {
  const c10::DeviceGuard guard(fl_.device());
  check_dev("allpairs_corr", fl_); check_dev("allpairs_corr", fr_);
  TORCH_CHECK(fl_.dim() == 4 && fl_.sizes() == fr_.sizes(), "allpairs_corr: fl, fr must be (B,C,H,W) alike");
  TORCH_CHECK(num_levels >= 1 && num_levels <= 8, "allpairs_corr: num_levels in [1,8]");
  Tensor fl = dense(fl_), fr = dense(fr_);
  const int64_t B = fl.size(0), C = fl.size(1), H = fl.size(2), W = fl.size(3);
  std::vector<Tensor> levels;
  std::vector<float*> ptrs;
  for (int64_t i = 0; i < num_levels; ++i) {
    levels.push_back(at::empty({B, H, W, W >> i}, fl.options()));
    ptrs.push_back(mp(levels.back()));
  }
  Tensor ws = at::empty({2, B, C, H, W}, fl.options());
  ok(fsmi_allpairs_corr(cp(fl), cp(fr), ptrs.data(), num_levels, B, C, H, W, mp(ws), stream_of(fl)),
     "allpairs_corr");
  return levels;
}

std::vector<Tensor> volume_pyramid(const Tensor& vol_, int64_t num_levels) {
  const c10::DeviceGuard guard(vol_.device());
  check_dev("volume_pyramid", vol_);
  TORCH_CHECK(vol_.dim() == 5, "volume_pyramid: vol must be (B,Cv,D,H,W)");
  TORCH_CHECK(num_levels >= 1 && num_levels <= 8, "volume_pyramid: num_levels in [1,8]");
  Tensor vol = dense(vol_);
  const int64_t B = vol.size(0), Cv = vol.size(1), D = vol.size(2), H = vol.size(3), W = vol.size(4);
  std::vector<Tensor> levels{vol};
  std::vector<float*> ptrs;
  for (int64_t i = 1; i < num_levels; ++i) {
    levels.push_back(at::empty({B, Cv, D >> i, H, W}, vol.options()));
    ptrs.push_back(mp(levels.back()));
  }
  if (num_levels > 1)
    ok(fsmi_volume_pyramid(cp(vol), ptrs.data(), num_levels, B, Cv, D, H, W, stream_of(vol)), "volume_pyramid");
  return levels;
}

Tensor geo_lookup(at::TensorList vol_levels, at::TensorList corr_levels, const Tensor& disp_, int64_t radius,
                  const c10::optional<Tensor>& coords_) {
  const int64_t L = vol_levels.size();
  TORCH_CHECK(L >= 1 && L <= 8 && (int64_t)corr_levels.size() == L, "geo_lookup: 1..8 levels of each pyramid");
  check_dev("geo_lookup", disp_);
  const c10::DeviceGuard guard(disp_.device());
  const Tensor& v0 = vol_levels[0];
  TORCH_CHECK(v0.dim() == 5, "geo_lookup: volume levels must be (B,Cv,D,H,W)");
  const int64_t B = v0.size(0), Cv = v0.size(1), D = v0.size(2), H = v0.size(3), W = v0.size(4);
  const int64_t W2 = corr_levels[0].size(-1);
  TORCH_CHECK(disp_.sizes() == at::IntArrayRef({B, 1, H, W}), "geo_lookup: disp ", disp_.sizes(),
              " vs volume (", B, ",1,", H, ",", W, ")");
  std::vector<const float*> pv, pc;
  for (int64_t i = 0; i < L; ++i) {
    check_dev("geo_lookup", vol_levels[i]); check_dev("geo_lookup", corr_levels[i]);
    TORCH_CHECK(vol_levels[i].sizes() == at::IntArrayRef({B, Cv, D >> i, H, W}) && vol_levels[i].is_contiguous(),
                "geo_lookup: volume level ", i, " must be contiguous (B,Cv,D>>i,H,W)");
    TORCH_CHECK(corr_levels[i].sizes() == at::IntArrayRef({B, H, W, W2 >> i}) && corr_levels[i].is_contiguous(),
                "geo_lookup: corr level ", i, " must be contiguous (B,H,W,W2>>i)");
    pv.push_back(cp(vol_levels[i]));
    pc.push_back(cp(corr_levels[i]));
  }
  Tensor disp = dense(disp_);
  const int64_t K = 2 * radius + 1;
  Tensor out = at::empty({B, L * K * (Cv + 1), H, W}, disp.options());
  Tensor coords;       // the reference's coords (core/geometry.py:57): any layout of B*H*W values
  if (coords_.has_value() && coords_->defined()) {
    check_dev("geo_lookup", *coords_);
    TORCH_CHECK(coords_->numel() == B * H * W, "geo_lookup: coords must hold B*H*W values");
    coords = dense(coords_->reshape({B, H, W}));
  }
  ok(fsmi_geo_lookup_coords(pv.data(), pc.data(), cp(disp), coords.defined() ? cp(coords) : nullptr, mp(out), L,
                            radius, B, Cv, D, H, W, W2, stream_of(disp)),
     "geo_lookup");
  return out;
}

Tensor bilinear_sampler_1d(const Tensor& img_, const Tensor& x_) {
  const c10::DeviceGuard guard(img_.device());
  check_dev("bilinear_sampler", img_); check_dev("bilinear_sampler", x_);
  TORCH_CHECK(img_.dim() == 4 && img_.size(2) == 1, "bilinear_sampler_1d: img must be (P,C,1,Lx)");
  const int64_t P = img_.size(0), C = img_.size(1), Lx = img_.size(3), K = x_.size(-1);
  TORCH_CHECK(x_.numel() == P * K, "bilinear_sampler_1d: x must hold (P,K) coordinates");
  Tensor img = dense(img_), x = dense(x_.reshape({P, K}));
  Tensor out = at::empty({P, C, 1, K}, img.options());
  ok(fsmi_bilinear_sampler_1d(cp(img), cp(x), mp(out), P, C, Lx, K, stream_of(img)), "bilinear_sampler");
  return out;
}

Tensor disparity_regression(const Tensor& prob_, int64_t maxdisp) {
  const c10::DeviceGuard guard(prob_.device());
  check_dev("disparity_regression", prob_);
  TORCH_CHECK(prob_.dim() == 4 && prob_.size(1) == maxdisp, "disparity_regression: prob must be (B,maxdisp,H,W)");
  Tensor prob = dense(prob_);
  const int64_t B = prob.size(0), D = prob.size(1), H = prob.size(2), W = prob.size(3);
  Tensor out = at::empty({B, 1, H, W}, prob.options());
  ok(fsmi_disparity_regression(cp(prob), mp(out), B, D, H, W, stream_of(prob)), "disparity_regression");
  return out;
}

Tensor softmax_regression(const Tensor& logits_) {
  const c10::DeviceGuard guard(logits_.device());
  check_dev("softmax_regression", logits_);
  TORCH_CHECK(logits_.dim() == 4, "softmax_regression: logits must be (B,D,H,W)");
  Tensor logits = dense(logits_);
  const int64_t B = logits.size(0), D = logits.size(1), H = logits.size(2), W = logits.size(3);
  Tensor out = at::empty({B, 1, H, W}, logits.options());
  ok(fsmi_softmax_regression(cp(logits), mp(out), B, D, H, W, stream_of(logits)), "softmax_regression");
  return out;
}

Tensor context_upsample(const Tensor& disp_, const Tensor& w_) {
  const c10::DeviceGuard guard(disp_.device());
  check_dev("context_upsample", disp_); check_dev("context_upsample", w_);
  TORCH_CHECK(disp_.dim() == 4 && disp_.size(1) == 1, "context_upsample: disp_low must be (B,1,h,w)");
  const int64_t B = disp_.size(0), h = disp_.size(2), w = disp_.size(3);
  TORCH_CHECK(w_.sizes() == at::IntArrayRef({B, 9, 4 * h, 4 * w}), "context_upsample: up_weights must be (B,9,4h,4w)");
  Tensor disp = dense(disp_), wt = dense(w_);
  Tensor out = at::empty({B, 4 * h, 4 * w}, disp.options());
  ok(fsmi_context_upsample(cp(disp), cp(wt), mp(out), B, h, w, stream_of(disp)), "context_upsample");
  return out;
}

Tensor softmax_context_upsample(const Tensor& disp_, const Tensor& logits_, double scale) {
  const c10::DeviceGuard guard(disp_.device());
  check_dev("softmax_context_upsample", disp_); check_dev("softmax_context_upsample", logits_);
  TORCH_CHECK(disp_.dim() == 4 && disp_.size(1) == 1, "softmax_context_upsample: disp_low must be (B,1,h,w)");
  const int64_t B = disp_.size(0), h = disp_.size(2), w = disp_.size(3);
  TORCH_CHECK(logits_.sizes() == at::IntArrayRef({B, 9, 4 * h, 4 * w}),
              "softmax_context_upsample: logits must be (B,9,4h,4w)");
  Tensor disp = dense(disp_), lg = dense(logits_);
  Tensor out = at::empty({B, 4 * h, 4 * w}, disp.options());
  ok(fsmi_softmax_context_upsample(cp(disp), cp(lg), mp(out), (float)scale, B, h, w, stream_of(disp)),
     "softmax_context_upsample");
  return out;
}

}  // namespace

TORCH_LIBRARY(fsmi, m) {
  m.def("gwc_volume(Tensor fl, Tensor fr, int maxdisp, int num_groups) -> Tensor");
  m.def("concat_volume(Tensor pl, Tensor pr, int maxdisp) -> Tensor");
  m.def("allpairs_corr(Tensor fl, Tensor fr, int num_levels) -> Tensor[]");
  // level 0 IS `vol` (the reference keeps the filtered volume as its level 0, core/geometry.py:29-36)
  m.def("volume_pyramid(Tensor(a -> *) vol, int num_levels) -> Tensor(a)[]");
  m.def("geo_lookup(Tensor[] vol_levels, Tensor[] corr_levels, Tensor disp, int radius, Tensor? coords=None) -> Tensor");
  m.def("bilinear_sampler_1d(Tensor img, Tensor x) -> Tensor");
  m.def("disparity_regression(Tensor prob, int maxdisp) -> Tensor");
  m.def("softmax_regression(Tensor logits) -> Tensor");
  m.def("context_upsample(Tensor disp_low, Tensor up_weights) -> Tensor");
  m.def("softmax_context_upsample(Tensor disp_low, Tensor logits, float scale=4.0) -> Tensor");
}

// ROCm builds of PyTorch expose HIP devices under the CUDA dispatch key
TORCH_LIBRARY_IMPL(fsmi, CUDA, m) {
  m.impl("gwc_volume", gwc_volume);
  m.impl("concat_volume", concat_volume);
  m.impl("allpairs_corr", allpairs_corr);
  m.impl("volume_pyramid", volume_pyramid);
  m.impl("geo_lookup", geo_lookup);
  m.impl("bilinear_sampler_1d", bilinear_sampler_1d);
  m.impl("disparity_regression", disparity_regression);
  m.impl("softmax_regression", softmax_regression);
  m.impl("context_upsample", context_upsample);
  m.impl("softmax_context_upsample", softmax_context_upsample);
}
