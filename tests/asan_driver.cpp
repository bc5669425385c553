// Host-side AddressSanitizer driver of the C-ABI (SURVEY §5 "race detection
// / sanitizers").  Linked with engine.hip's host code compiled under
// -Xarch_host -fsanitize=address (device code unsanitized: GPU ASan is not
// available), see nanodecoder_amd/build.py build_asan().  Test
// infrastructure, run by tests/test_asan.py.
//
//   asan_driver                 argument validation and the no-device error
//                               paths of every entry point (CPU)
//   asan_driver --gpu W.bin     + the full lifecycle on a device: create,
//                               weight errors, finalize errors, finalize,
//                               translate (greedy, beam) argument errors and
//                               calls, destroy
//
// W.bin: u32 count, then per tensor u32 name length, name, u32 ndim, i64
// dims[ndim], f32 data (tests/test_asan.py writes it from synth.make_weights).
// Exit status: number of failed checks (0 = pass).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <unistd.h>
#include <string>
#include <vector>

#include "../include/nanodec.h"

static int g_fail = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      ++g_fail;                                                              \
      fprintf(stderr, "FAIL %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, #cond, nd_last_error()); \
    }                                                                        \
  } while (0)

static nd_config good_config() {
  nd_config c{};
  c.encoder_type = ND_ENC_TRANSFORMER;
  c.enc_layers = 3;
  c.dec_layers = 3;
  c.d_model = 256;
  c.heads = 8;
  c.d_ff = 2048;
  c.vocab = 8;
  c.rnn_hidden = 128;
  c.position_encoding = 1;
  c.pad_idx = 1;
  c.bos_idx = 2;
  c.eos_idx = 3;
  c.max_batch = 4;
  c.max_src_len = 512;
  c.max_steps = 12;
  c.max_beam = 2;
  c.device = 0;
  c.self_attn_type = ND_SELF_SCALED_DOT;
  return c;
}

struct Tensor {
  std::string name;
  std::vector<int64_t> shape;
  std::vector<float> data;
};

static bool read_weights(const char* path, std::vector<Tensor>& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  uint32_t n = 0;
  bool ok = fread(&n, 4, 1, f) == 1;
  for (uint32_t i = 0; ok && i < n; ++i) {
    Tensor t;
    uint32_t len = 0, nd = 0;
    ok = fread(&len, 4, 1, f) == 1 && len < 4096;
    if (!ok) break;
    t.name.resize(len);
    ok = fread(&t.name[0], 1, len, f) == len && fread(&nd, 4, 1, f) == 1 && nd <= 4;
    if (!ok) break;
    t.shape.resize(nd);
    size_t numel = 1;
    ok = fread(t.shape.data(), 8, nd, f) == nd;
    for (auto d : t.shape) numel *= (size_t)d;
    t.data.resize(numel);
    ok = ok && fread(t.data.data(), 4, numel, f) == numel;
    out.push_back(std::move(t));
  }
  fclose(f);
  return ok;
}

// every entry point with a null context / null arguments: ND_ERR_ARG, no crash
static void null_paths() {
  nd_ctx* c = reinterpret_cast<nd_ctx*>(0x1);
  CHECK(nd_create(nullptr, &c) == ND_ERR_ARG);
  nd_config cfg = good_config();
  CHECK(nd_create(&cfg, nullptr) == ND_ERR_ARG);
  float buf[4] = {0, 0, 0, 0};
  int64_t shape[1] = {4};
  CHECK(nd_load_weight(nullptr, "encoder.linear.bias", buf, shape, 1) == ND_ERR_ARG);
  CHECK(nd_finalize(nullptr) == ND_ERR_ARG);
  int32_t i4[4] = {0, 0, 0, 0};
  CHECK(nd_translate_greedy(nullptr, buf, i4, i4, 1, 4, 1, 0, i4, buf, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_beam(nullptr, buf, i4, i4, 1, 4, 1, 1, 0.f, 1, 0, i4, buf, i4, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_encode(nullptr, buf, i4, i4, 1, 4, buf, nullptr) == ND_ERR_ARG);
  CHECK(nd_set_graphs(nullptr, 1) == ND_ERR_ARG);
  CHECK(nd_set_ctx_path(nullptr, 0) == ND_ERR_ARG);
  CHECK(nd_set_exact_fp32(nullptr, 1) == ND_ERR_ARG);
  CHECK(nd_set_timing(nullptr, 1) == ND_ERR_ARG);
  CHECK(nd_set_kernel_stamps(nullptr, 1) == ND_ERR_ARG);
  CHECK(nd_take_overflow(nullptr, i4, nullptr) == ND_ERR_ARG);
  float f = 0.f;
  int32_t k = 0;
  CHECK(nd_kernel_stamps(nullptr, &f, &k) == ND_ERR_ARG);
  CHECK(nd_last_timing(nullptr, &f, &f) == ND_ERR_ARG);
  CHECK(nd_stream(nullptr) == nullptr);
  CHECK(nd_gemm_routes(nullptr, 4, 0) == ND_ERR_ARG);
  int64_t routes[ND_ROUTE_N + 2];
  CHECK(nd_gemm_routes(routes, ND_ROUTE_N + 2, 1) == ND_OK);
  char small[3];
  CHECK(nd_switches(small, (int32_t)sizeof small) >= 0 && strlen(small) < sizeof small);
  CHECK(nd_switches(nullptr, 0) >= 0);
  nd_destroy(nullptr);
  CHECK(strlen(nd_version()) > 0);
  CHECK(strlen(nd_last_error()) > 0);
}

// invalid configurations: rejected before any device call, *out left null
static void config_paths() {
  struct Bad {
    const char* what;
    void (*mut)(nd_config&);
  } bad[] = {
      {"d_model", [](nd_config& c) { c.d_model = 128; }},
      {"heads", [](nd_config& c) { c.heads = 4; }},
      {"d_ff", [](nd_config& c) { c.d_ff = 100; }},
      {"d_ff0", [](nd_config& c) { c.d_ff = 0; }},
      {"vocab small", [](nd_config& c) { c.vocab = 3; }},
      {"vocab large", [](nd_config& c) { c.vocab = 33; }},
      {"src len", [](nd_config& c) { c.max_src_len = 513; }},
      {"src len 0", [](nd_config& c) { c.max_src_len = 0; }},
      {"steps", [](nd_config& c) { c.max_steps = 513; }},
      {"beam", [](nd_config& c) { c.max_beam = 9; }},
      {"batch", [](nd_config& c) { c.max_batch = 0; }},
      {"layers", [](nd_config& c) { c.dec_layers = 0; }},
      {"encoder", [](nd_config& c) { c.encoder_type = 5; }},
      {"rnn", [](nd_config& c) { c.encoder_type = ND_ENC_NANO; c.rnn_hidden = 64; }},
      {"self attn", [](nd_config& c) { c.self_attn_type = 9; }},
  };
  for (const auto& b : bad) {
    nd_config cfg = good_config();
    b.mut(cfg);
    nd_ctx* c = reinterpret_cast<nd_ctx*>(0x1);
    const int rc = nd_create(&cfg, &c);
    if (rc != ND_ERR_ARG || c != nullptr) {
      ++g_fail;
      fprintf(stderr, "FAIL config %s: rc %d\n", b.what, rc);
    }
  }
}

static void gpu_lifecycle(const char* wpath) {
  std::vector<Tensor> W;
  CHECK(read_weights(wpath, W));
  if (W.empty()) return;
  nd_config cfg = good_config();
  cfg.position_encoding = 0;  // as the weights file has it
  for (const auto& t : W) cfg.position_encoding |= t.name == "decoder.embeddings.make_embedding.pe.pe";
  nd_ctx* c = nullptr;
  CHECK(nd_create(&cfg, &c) == ND_OK && c != nullptr);
  if (!c) return;
  // weight errors
  float v[256] = {0};
  int64_t s1[1] = {256}, s2[2] = {256, 1}, bad1[1] = {255};
  CHECK(nd_load_weight(c, "no.such.weight", v, s1, 1) == ND_ERR_WEIGHT);
  CHECK(nd_load_weight(c, "encoder.linear.bias", v, s2, 2) == ND_ERR_WEIGHT);    // rank
  CHECK(nd_load_weight(c, "encoder.linear.bias", v, bad1, 1) == ND_ERR_WEIGHT);  // shape
  CHECK(nd_load_weight(c, "encoder.linear.bias", nullptr, s1, 1) == ND_ERR_ARG);
  CHECK(nd_load_weight(c, "decoder.transformer_layers.0.self_attn.mask", v, s1, 1) == ND_OK);  // ignored buffer
  CHECK(nd_finalize(c) == ND_ERR_WEIGHT);  // nothing loaded yet
  // state errors
  float* d_sig = nullptr;
  int32_t *d_len = nullptr, *d_tok = nullptr, *d_ln = nullptr;
  float* d_sc = nullptr;
  const int B = 4, T = 512, S = 12;
  CHECK(hipMalloc(&d_sig, (size_t)B * T * 4) == hipSuccess);
  CHECK(hipMalloc(&d_len, B * 4) == hipSuccess);
  CHECK(hipMalloc(&d_tok, (size_t)B * 2 * S * 4) == hipSuccess);
  CHECK(hipMalloc(&d_ln, B * 2 * 4) == hipSuccess);
  CHECK(hipMalloc(&d_sc, B * 2 * 4) == hipSuccess);
  std::vector<float> sig((size_t)B * T);
  for (size_t i = 0; i < sig.size(); ++i) sig[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  std::vector<int32_t> len(B, T);
  CHECK(hipMemcpy(d_sig, sig.data(), sig.size() * 4, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(hipMemcpy(d_len, len.data(), B * 4, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T, S, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_STATE);
  for (const auto& t : W)
    CHECK(nd_load_weight(c, t.name.c_str(), t.data.data(), t.shape.data(), (int)t.shape.size()) == ND_OK);
  CHECK(nd_finalize(c) == ND_OK);
  // call argument errors
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, 0, T, S, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B + 1, T, S, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T + 1, S, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T, S + 1, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_greedy(c, nullptr, d_len, d_len, B, T, S, 0, d_tok, d_sc, nullptr, nullptr) == ND_ERR_ARG);
  CHECK(nd_translate_beam(c, d_sig, d_len, d_len, B, T, 3, 1, 0.f, S, 0, d_tok, d_sc, d_ln, nullptr, nullptr) ==
        ND_ERR_ARG);  // beam > max_beam
  CHECK(nd_translate_beam(c, d_sig, d_len, d_len, B, T, 2, 3, 0.f, S, 0, d_tok, d_sc, d_ln, nullptr, nullptr) ==
        ND_ERR_ARG);  // n_best > beam
  CHECK(nd_set_ctx_path(c, 2) == ND_ERR_ARG);
  // calls (graphs on, then off; split and exact products)
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T, S, 2, d_tok, d_sc, nullptr, nullptr) == ND_OK);
  CHECK(nd_translate_beam(c, d_sig, d_len, d_len, B, T, 2, 2, 0.f, S, 0, d_tok, d_sc, d_ln, nullptr, nullptr) ==
        ND_OK);
  CHECK(nd_set_exact_fp32(c, 1) == ND_OK);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T, S, 2, d_tok, d_sc, nullptr, nullptr) == ND_OK);
  CHECK(nd_set_exact_fp32(c, 0) == ND_OK);
  CHECK(nd_set_graphs(c, 0) == ND_OK);
  CHECK(nd_translate_greedy(c, d_sig, d_len, d_len, B, T - 64, S, 2, d_tok, d_sc, nullptr, nullptr) == ND_OK);
  int32_t* d_ov = nullptr;
  CHECK(hipMalloc(&d_ov, 4) == hipSuccess);
  CHECK(nd_take_overflow(c, d_ov, nullptr) == ND_OK);
  CHECK(hipDeviceSynchronize() == hipSuccess);
  std::vector<int32_t> tok((size_t)B * S);
  CHECK(hipMemcpy(tok.data(), d_tok, tok.size() * 4, hipMemcpyDeviceToHost) == hipSuccess);
  for (int32_t t : tok) CHECK(t >= 0 && t < cfg.vocab);
  nd_destroy(c);
  for (void* p : {(void*)d_sig, (void*)d_len, (void*)d_tok, (void*)d_ln, (void*)d_sc, (void*)d_ov}) (void)hipFree(p);
}

int main(int argc, char** argv) {
  null_paths();
  config_paths();
  if (argc > 2 && strcmp(argv[1], "--gpu") == 0) {
    gpu_lifecycle(argv[2]);
  } else {
    // no device here: a valid configuration fails in the HIP runtime, cleanly
    nd_config cfg = good_config();
    nd_ctx* c = reinterpret_cast<nd_ctx*>(0x1);
    const int rc = nd_create(&cfg, &c);
    CHECK(rc == ND_ERR_HIP && c == nullptr);
  }
  printf("asan_driver: %d failed checks\n", g_fail);
  if (argc > 2) {
    // every context and buffer of ours is released above; skip the HIP
    // runtime's own static teardown, whose late host frees trip ASan's device
    // allocator check ("dev_runtime_unloaded_") on this ROCm
    fflush(stdout);
    fflush(stderr);
    _exit(g_fail);
  }
  return g_fail;
}
