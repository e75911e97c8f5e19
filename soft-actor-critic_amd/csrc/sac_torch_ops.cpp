// sac_torch_ops.cpp — PyTorch-ROCm custom ops over the C ABI (include/sac_engine.h).
//
// TORCH_LIBRARY(sac_hip): the operator boundary SURVEY.md §8(b) names for the
// hot path.  Every op launches on the caller's CURRENT HIP stream
// (torch.cuda.current_stream(): ROCm PyTorch's HIP stream masquerading as the
// "cuda" device type), never synchronises the host, allocates its
// outputs from the PyTorch caching allocator, and is capturable by
// torch.cuda.graph.  Meta kernels give the output shapes (fake tensors).
//
//   replay_push          ReplayBuffer.push            (reference sac/replay_buffer.py:21-30)
//   replay_gather        ReplayBuffer.sample +        (replay_buffer.py:32-39,
//                        SAC.sample_batch stacking     sac/agent.py:166-193)
//   replay_sample        the index draw of random.sample (replay_buffer.py:39)
//   replay_sample_gather sampler + gather in one kernel
//   train_step           SAC.training_step            (sac/agent.py:302-327)
//   train_graph          a loop of training_step      (sac/agent.py:361-364), hipGraph-replayed
//   policy_act           SAC.select_action            (sac/agent.py:149-156; models.py:79-92)
//
// Replay storage is ONE fp32 tensor per buffer; `layout` = [capacity, obs_dim,
// act_dim, row_stride, off_obs, off_act, off_rew, off_next_obs, off_done]
// (offsets in floats from storage.data_ptr(); row_stride 0 = struct-of-arrays).
// Engine state: `engine` is the sac_engine* handle (int64) from
// sac_engine_create; `state` lists the 16 caller-owned tensors the step reads
// and writes (sac_engine_buffers order) so the op's mutation is declared.
//
// The ops do not link libsac_engine.so: bind_engine_library(path) dlopens the
// library the Python side loaded (the same file, hence the same instance as the
// ctypes handle's owner, also for the diagnostic -DSAC_STAMPS build) and
// resolves the entry points once.
#include <dlfcn.h>

#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "sac_engine.h"

namespace {

constexpr int64_t kStateTensors = 16;
using Guard = c10::hip::HIPGuardMasqueradingAsCUDA;

// the C ABI entry points the ops call, resolved by bind_engine_library
struct EngineApi {
  decltype(&sac_last_error) last_error = nullptr;
  decltype(&sac_replay_push) replay_push = nullptr;
  decltype(&sac_replay_gather) replay_gather = nullptr;
  decltype(&sac_replay_sample_indices) replay_sample_indices = nullptr;
  decltype(&sac_replay_sample_gather) replay_sample_gather = nullptr;
  decltype(&sac_engine_train) engine_train = nullptr;
  decltype(&sac_engine_train_graph) engine_train_graph = nullptr;
  decltype(&sac_policy_act) policy_act = nullptr;
};
EngineApi g_api;
std::string g_bound_path;

template <typename F>
void resolve(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  TORCH_CHECK(f != nullptr, "libsac_engine lacks ", name);
}

void bind_engine_library(c10::string_view path_) {
  const std::string path(path_.data(), path_.size());
  if (g_api.engine_train && path == g_bound_path) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  TORCH_CHECK(h != nullptr, "cannot load ", path, ": ", dlerror());
  EngineApi a;
  resolve(h, "sac_last_error", a.last_error);
  resolve(h, "sac_replay_push", a.replay_push);
  resolve(h, "sac_replay_gather", a.replay_gather);
  resolve(h, "sac_replay_sample_indices", a.replay_sample_indices);
  resolve(h, "sac_replay_sample_gather", a.replay_sample_gather);
  resolve(h, "sac_engine_train", a.engine_train);
  resolve(h, "sac_engine_train_graph", a.engine_train_graph);
  resolve(h, "sac_policy_act", a.policy_act);
  g_api = a;
  g_bound_path = path;
}

const EngineApi& api() {
  TORCH_CHECK(g_api.engine_train != nullptr,
              "torch.ops.sac_hip: engine library not bound (call sac._engine.ops(), which binds libsac_engine.so)");
  return g_api;
}

void* stream_of(const at::Tensor& t) {
  return static_cast<void*>(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream());
}

void check_rc(int rc) {
  // SAC_E_NOT_ENOUGH is the reference's ValueError (replay_buffer.py:35-38)
  if (rc == SAC_OK) return;
  TORCH_CHECK_VALUE(rc != SAC_E_NOT_ENOUGH, api().last_error());
  TORCH_CHECK(false, "libsac_engine error ", rc, ": ", api().last_error());
}

void check_f32(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a HIP device tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, what, " must be float32");
  TORCH_CHECK(t.is_contiguous(), what, " must be contiguous");
}

struct Replay {
  sac_replay d;
  int64_t obs, act;
};

Replay make_replay(const at::Tensor& storage, const at::Tensor& state, at::IntArrayRef layout) {
  TORCH_CHECK(layout.size() == 9, "replay layout must have 9 entries");
  check_f32(storage, "replay storage");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kLong && state.numel() >= 3 && state.is_contiguous(),
              "replay state must be a contiguous int64 device tensor of >= 3 entries");
  TORCH_CHECK(state.device() == storage.device(), "replay state and storage on different devices");
  const int64_t cap = layout[0], O = layout[1], A = layout[2], stride = layout[3];
  TORCH_CHECK(cap >= 1 && O >= 1 && A >= 1 && stride >= 0, "bad replay layout");
  const int64_t width[5] = {O, A, 1, O, 1};
  const int64_t n = storage.numel();
  for (int f = 0; f < 5; ++f) {
    const int64_t off = layout[4 + f];
    const int64_t end = stride ? off + (cap - 1) * stride + width[f] : off + cap * width[f];
    TORCH_CHECK(off >= 0 && end <= n, "replay field ", f, " exceeds the storage tensor");
    if (stride) TORCH_CHECK(width[f] <= stride, "record stride narrower than a field");
  }
  float* base = storage.data_ptr<float>();
  Replay r;
  r.d.obs = base + layout[4];
  r.d.act = base + layout[5];
  r.d.rew = base + layout[6];
  r.d.next_obs = base + layout[7];
  r.d.done = base + layout[8];
  r.d.capacity = cap;
  r.d.obs_dim = static_cast<int32_t>(O);
  r.d.act_dim = static_cast<int32_t>(A);
  r.d.state = state.data_ptr<int64_t>();
  r.d.row_stride = stride;
  r.obs = O;
  r.act = A;
  return r;
}

sac_engine* engine_of(int64_t handle, const at::TensorList& state, const at::Tensor& like) {
  TORCH_CHECK(handle != 0, "null engine handle");
  TORCH_CHECK(static_cast<int64_t>(state.size()) == kStateTensors, "engine state must list ", kStateTensors,
              " tensors (sac_engine_buffers order)");
  for (const auto& t : state)
    TORCH_CHECK(t.is_cuda() && t.device() == like.device(), "engine state tensor not on the replay's device");
  return reinterpret_cast<sac_engine*>(handle);
}

// ---------------------------------------------------------------- replay
void replay_push(at::Tensor& storage, at::Tensor& state, at::IntArrayRef layout, const at::Tensor& rows,
                 int64_t size, int64_t pos) {
  Replay r = make_replay(storage, state, layout);
  check_f32(rows, "rows");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 2 * r.obs + r.act + 2, "rows must be [n][2*obs+act+2]");
  TORCH_CHECK(rows.device() == storage.device(), "rows on a different device");
  if (rows.size(0) == 0) return;
  Guard g(storage.device());
  check_rc(api().replay_push(&r.d, rows.data_ptr<float>(), rows.size(0), size, pos, stream_of(storage)));
}

std::vector<at::Tensor> empty_batch(const at::Tensor& like, int64_t B, int64_t O, int64_t A) {
  auto o = like.options().dtype(at::kFloat);
  return {at::empty({B, O}, o), at::empty({B, A}, o), at::empty({B}, o), at::empty({B, O}, o), at::empty({B}, o)};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> replay_gather(
    const at::Tensor& storage, const at::Tensor& state, at::IntArrayRef layout, const at::Tensor& indices) {
  Replay r = make_replay(storage, state, layout);
  TORCH_CHECK(indices.is_cuda() && indices.scalar_type() == at::kInt && indices.dim() == 1 && indices.is_contiguous(),
              "indices must be a contiguous 1-D int32 device tensor");
  const int64_t B = indices.size(0);
  auto out = empty_batch(storage, B, r.obs, r.act);
  if (B) {
    Guard g(storage.device());
    check_rc(api().replay_gather(&r.d, indices.data_ptr<int32_t>(), static_cast<int32_t>(B), out[0].data_ptr<float>(),
                               out[1].data_ptr<float>(), out[2].data_ptr<float>(), out[3].data_ptr<float>(),
                               out[4].data_ptr<float>(), stream_of(storage)));
  }
  return {out[0], out[1], out[2], out[3], out[4]};
}

at::Tensor replay_sample(const at::Tensor& storage, const at::Tensor& state, at::IntArrayRef layout, int64_t batch,
                         int64_t seed, int64_t step) {
  Replay r = make_replay(storage, state, layout);
  TORCH_CHECK(batch >= 1 && batch <= r.d.capacity, "batch must be in [1, capacity]");
  auto idx = at::empty({batch}, storage.options().dtype(at::kInt));
  Guard g(storage.device());
  check_rc(api().replay_sample_indices(&r.d, static_cast<int32_t>(batch), static_cast<uint64_t>(seed),
                                     static_cast<uint64_t>(step), idx.data_ptr<int32_t>(), stream_of(storage)));
  return idx;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> replay_sample_gather(
    const at::Tensor& storage, const at::Tensor& state, at::IntArrayRef layout, int64_t batch, int64_t seed,
    int64_t step) {
  Replay r = make_replay(storage, state, layout);
  TORCH_CHECK(batch >= 1 && batch <= r.d.capacity, "batch must be in [1, capacity]");
  auto idx = at::empty({batch}, storage.options().dtype(at::kInt));
  auto out = empty_batch(storage, batch, r.obs, r.act);
  Guard g(storage.device());
  check_rc(api().replay_sample_gather(&r.d, static_cast<int32_t>(batch), static_cast<uint64_t>(seed),
                                    static_cast<uint64_t>(step), idx.data_ptr<int32_t>(), out[0].data_ptr<float>(),
                                    out[1].data_ptr<float>(), out[2].data_ptr<float>(), out[3].data_ptr<float>(),
                                    out[4].data_ptr<float>(), stream_of(storage)));
  return {idx, out[0], out[1], out[2], out[3], out[4]};
}

// ---------------------------------------------------------------- learner
void train_step(int64_t engine, at::TensorList state, const at::Tensor& storage, const at::Tensor& rstate,
                at::IntArrayRef layout, int64_t n_steps, const std::optional<at::Tensor>& indices,
                const std::optional<at::Tensor>& eps) {
  Replay r = make_replay(storage, rstate, layout);
  sac_engine* e = engine_of(engine, state, storage);
  TORCH_CHECK(n_steps >= 0, "n_steps must be >= 0");
  const int32_t* ip = nullptr;
  const float* ep = nullptr;
  if (indices && indices->defined()) {
    const auto& t = *indices;
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.dim() == 2 &&
                    t.size(0) >= n_steps,
                "indices must be a contiguous [n_steps][batch] int32 device tensor");
    ip = t.data_ptr<int32_t>();
  }
  if (eps && eps->defined()) {
    const auto& t = *eps;
    check_f32(t, "eps");
    TORCH_CHECK(t.dim() == 4 && t.size(0) >= n_steps && t.size(1) == 2 && t.size(3) == r.act,
                "eps must be [n_steps][2][batch][act_dim]");
    ep = t.data_ptr<float>();
  }
  if (!n_steps) return;
  Guard g(storage.device());
  check_rc(api().engine_train(e, &r.d, static_cast<int32_t>(n_steps), ip, ep, stream_of(storage)));
}

void train_graph(int64_t engine, at::TensorList state, const at::Tensor& storage, const at::Tensor& rstate,
                 at::IntArrayRef layout, int64_t n_steps, int64_t chunk) {
  Replay r = make_replay(storage, rstate, layout);
  sac_engine* e = engine_of(engine, state, storage);
  TORCH_CHECK(n_steps >= 0 && chunk >= 1, "n_steps >= 0 and chunk >= 1");
  Guard g(storage.device());
  check_rc(api().engine_train_graph(e, &r.d, static_cast<int32_t>(n_steps), static_cast<int32_t>(chunk),
                                  stream_of(storage)));
}

std::tuple<at::Tensor, at::Tensor> policy_act(int64_t engine, const at::Tensor& obs, const std::optional<at::Tensor>& eps,
                                              int64_t act_dim, bool want_log_pi) {
  TORCH_CHECK(engine != 0, "null engine handle");
  check_f32(obs, "obs");
  TORCH_CHECK(obs.dim() == 2, "obs must be [n][obs_dim]");
  const int64_t n = obs.size(0);
  const float* ep = nullptr;
  if (eps && eps->defined()) {
    check_f32(*eps, "eps");
    TORCH_CHECK(eps->dim() == 2 && eps->size(0) == n && eps->size(1) == act_dim, "eps must be [n][act_dim]");
    ep = eps->data_ptr<float>();
  }
  auto o = obs.options();
  at::Tensor act = at::empty({n, act_dim}, o);
  at::Tensor lp = at::empty({(want_log_pi && ep) ? n : 0}, o);
  if (n) {
    Guard g(obs.device());
    check_rc(api().policy_act(reinterpret_cast<sac_engine*>(engine), obs.data_ptr<float>(), static_cast<int32_t>(n), ep,
                            act.data_ptr<float>(), lp.numel() ? lp.data_ptr<float>() : nullptr, stream_of(obs)));
  }
  return {act, lp};
}

// ---------------------------------------------------------------- meta (shapes only)
void replay_push_meta(at::Tensor&, at::Tensor&, at::IntArrayRef, const at::Tensor&, int64_t, int64_t) {}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> replay_gather_meta(
    const at::Tensor& storage, const at::Tensor&, at::IntArrayRef layout, const at::Tensor& indices) {
  auto o = empty_batch(storage, indices.size(0), layout[1], layout[2]);
  return {o[0], o[1], o[2], o[3], o[4]};
}

at::Tensor replay_sample_meta(const at::Tensor& storage, const at::Tensor&, at::IntArrayRef, int64_t batch, int64_t,
                              int64_t) {
  return at::empty({batch}, storage.options().dtype(at::kInt));
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> replay_sample_gather_meta(
    const at::Tensor& storage, const at::Tensor&, at::IntArrayRef layout, int64_t batch, int64_t, int64_t) {
  auto o = empty_batch(storage, batch, layout[1], layout[2]);
  return {at::empty({batch}, storage.options().dtype(at::kInt)), o[0], o[1], o[2], o[3], o[4]};
}

void train_step_meta(int64_t, at::TensorList, const at::Tensor&, const at::Tensor&, at::IntArrayRef, int64_t,
                     const std::optional<at::Tensor>&, const std::optional<at::Tensor>&) {}

void train_graph_meta(int64_t, at::TensorList, const at::Tensor&, const at::Tensor&, at::IntArrayRef, int64_t,
                      int64_t) {}

std::tuple<at::Tensor, at::Tensor> policy_act_meta(int64_t, const at::Tensor& obs, const std::optional<at::Tensor>& eps,
                                                   int64_t act_dim, bool want_log_pi) {
  const int64_t n = obs.size(0);
  const bool lp = want_log_pi && eps && eps->defined();
  return {at::empty({n, act_dim}, obs.options()), at::empty({lp ? n : 0}, obs.options())};
}

}  // namespace

TORCH_LIBRARY(sac_hip, m) {
  m.def("bind_engine_library(str path) -> ()", &bind_engine_library);
  m.def("replay_push(Tensor(a!) storage, Tensor(b!) state, int[] layout, Tensor rows, int size, int pos) -> ()");
  m.def("replay_gather(Tensor storage, Tensor state, int[] layout, Tensor indices) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("replay_sample(Tensor storage, Tensor state, int[] layout, int batch, int seed, int step) -> Tensor");
  m.def("replay_sample_gather(Tensor storage, Tensor state, int[] layout, int batch, int seed, int step) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("train_step(int engine, Tensor(a!)[] state, Tensor storage, Tensor replay_state, int[] layout, "
        "int n_steps, Tensor? indices=None, Tensor? eps=None) -> ()");
  m.def("train_graph(int engine, Tensor(a!)[] state, Tensor storage, Tensor replay_state, int[] layout, "
        "int n_steps, int chunk) -> ()");
  m.def("policy_act(int engine, Tensor obs, Tensor? eps, int act_dim, bool want_log_pi=False) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(sac_hip, CUDA, m) {
  m.impl("replay_push", &replay_push);
  m.impl("replay_gather", &replay_gather);
  m.impl("replay_sample", &replay_sample);
  m.impl("replay_sample_gather", &replay_sample_gather);
  m.impl("train_step", &train_step);
  m.impl("train_graph", &train_graph);
  m.impl("policy_act", &policy_act);
}

TORCH_LIBRARY_IMPL(sac_hip, Meta, m) {
  m.impl("replay_push", &replay_push_meta);
  m.impl("replay_gather", &replay_gather_meta);
  m.impl("replay_sample", &replay_sample_meta);
  m.impl("replay_sample_gather", &replay_sample_gather_meta);
  m.impl("train_step", &train_step_meta);
  m.impl("train_graph", &train_graph_meta);
  m.impl("policy_act", &policy_act_meta);
}
