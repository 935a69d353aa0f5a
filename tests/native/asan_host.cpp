// Host-side AddressSanitizer driver for libeosv's C++ glue (sanitizers on host code only;
// GPU ASan is not available on this pool).  Built by `make -C <pkg>/csrc asan` from objects compiled
// with `-Xarch_host -fsanitize=address`, so the device code is unchanged and no GPU is needed.
//
//   asan_host plan N_WAY K_SHOT SEED N_EPISODES SIZE...   the plan service (eosv_plan_episodes),
//                                                        prints the plans as one line of ints
//   asan_host args                                       every entry point's argument validation:
//                                                        null / negative / oversize arguments must
//                                                        return an error code with a message, and
//                                                        nothing may touch memory it does not own
// Exit status 0 = every check held (ASan aborts with its own report otherwise).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "eosv.h"

static int fails = 0;

static void expect_err(int rc, const char* what) {
  const char* msg = eosv_last_error();
  if (rc >= 0 || !msg || !*msg) {
    std::printf("FAIL %s: rc %d msg '%s'\n", what, rc, msg ? msg : "(null)");
    ++fails;
  }
}

static int plan(int argc, char** argv) {
  if (argc < 7) return 2;
  const int n_way = std::atoi(argv[2]), k_shot = std::atoi(argv[3]);
  const unsigned long long seed = std::strtoull(argv[4], nullptr, 10);
  const int E = std::atoi(argv[5]);
  std::vector<int32_t> sizes;
  for (int i = 6; i < argc; ++i) sizes.push_back(std::atoi(argv[i]));
  std::vector<int32_t> cls((size_t)E * n_way), q((size_t)E * 2), sup((size_t)E * n_way * k_shot);
  const int rc = eosv_plan_episodes(sizes.data(), (int)sizes.size(), n_way, k_shot, seed, E, cls.data(), q.data(),
                                    sup.data());
  if (rc) {
    std::printf("ERR %d %s\n", rc, eosv_last_error());
    return 0;
  }
  for (int e = 0; e < E; ++e) {
    for (int i = 0; i < n_way; ++i) std::printf("%d ", cls[(size_t)e * n_way + i]);
    std::printf("%d %d ", q[2 * e], q[2 * e + 1]);
    for (int i = 0; i < n_way * k_shot; ++i) std::printf("%d ", sup[(size_t)e * n_way * k_shot + i]);
  }
  std::printf("\n");
  return 0;
}

static int args() {
  int32_t sizes[3] = {4, 4, 4}, out[64];
  expect_err(eosv_plan_episodes(nullptr, 3, 2, 1, 0, 1, out, out, out), "plan: null sizes");
  expect_err(eosv_plan_episodes(sizes, 3, 4, 1, 0, 1, out, out, out), "plan: n_way > classes");
  expect_err(eosv_plan_episodes(sizes, 3, 2, 4, 0, 1, out, out, out), "plan: k_shot + 1 > videos");
  expect_err(eosv_plan_episodes(sizes, 3, 0, 1, 0, 1, out, out, out), "plan: n_way 0");
  expect_err(eosv_plan_episodes(sizes, 3, 2, -1, 0, 1, out, out, out), "plan: negative k_shot");
  expect_err(eosv_plan_episodes(sizes, 3, 2, 1, 0, -1, out, out, out), "plan: negative episodes");

  expect_err(eosv_create(nullptr, nullptr), "create: null");
  eosv_desc d{};
  d.arch = 34;
  d.dtype = EOSV_F32;
  d.height = d.width = 224;
  d.max_frames = 16;
  d.num_classes = 64;
  eosv_handle* h = nullptr;
  expect_err(eosv_create(&d, &h), "create: unknown arch");
  d.arch = EOSV_ARCH_R18;
  d.dtype = 7;
  expect_err(eosv_create(&d, &h), "create: unknown dtype");
  d.dtype = EOSV_F32;
  d.height = 0;
  expect_err(eosv_create(&d, &h), "create: zero height");
  d.height = 224;
  d.max_frames = 0;
  expect_err(eosv_create(&d, &h), "create: zero max_frames");

  expect_err(eosv_load_weights(nullptr, nullptr, nullptr, nullptr, 0), "load_weights: null handle");
  expect_err(eosv_backbone_forward(nullptr, nullptr, 1, nullptr, nullptr), "forward: null handle");
  expect_err(eosv_fc_forward(nullptr, nullptr, 1, nullptr, nullptr), "fc: null handle");
  expect_err(eosv_clip_embed(nullptr, nullptr, nullptr, 1, 4096, 1, nullptr, nullptr), "clip_embed: D > 2048");
  expect_err(eosv_clip_embed(nullptr, nullptr, nullptr, -1, 512, 1, nullptr, nullptr), "clip_embed: negative clips");
  expect_err(eosv_segment_mean(nullptr, 4, 0, 512, nullptr, nullptr), "segment_mean: seg_len 0");
  expect_err(eosv_match(nullptr, nullptr, nullptr, nullptr, nullptr, 3, 512, 0, nullptr, nullptr, nullptr),
             "match: null");
  expect_err(eosv_match((const float*)out, (const float*)out, out, out, out, 1, 512, 9, (int64_t*)out, nullptr,
                        nullptr),
             "match: unknown kind");
  expect_err(eosv_segment_match(nullptr, 8, nullptr, 16, 2048, 0.1f, 1.f, nullptr, nullptr, nullptr),
             "segment_match: null");
  expect_err(eosv_segment_match_episodes(nullptr, 0, 8, nullptr, 16, 2048, 0.1f, 1.f, nullptr, nullptr, nullptr),
             "segment_match_episodes: zero episodes");
  expect_err(eosv_temporal_smooth(nullptr, 4, 4, 0.1f, 1.f, nullptr, nullptr), "temporal_smooth: null");
  const float mean[3] = {0.5f, 0.5f, 0.5f}, stdv[3] = {0.2f, 0.2f, 0.2f};
  expect_err(eosv_normalize_frames(nullptr, 1, 256, 340, 300, mean, stdv, nullptr, nullptr),
             "normalize: crop > frame");
  expect_err(eosv_crop_normalize_frames(nullptr, 1, 256, 340, 224, 40, 0, 0, mean, stdv, nullptr, nullptr),
             "crop_normalize: window outside");
  expect_err(eosv_synth_frames(nullptr, 1, 224, 224, nullptr, nullptr), "synth: null");
  expect_err(eosv_profile_enable(nullptr, 1), "profile_enable: null");
  expect_err(eosv_profile_read(nullptr, nullptr, nullptr, nullptr, 4), "profile_read: null");
  if (eosv_feature_dim(nullptr) != -1) {
    std::printf("FAIL feature_dim(null)\n");
    ++fails;
  }
  if (eosv_device_bytes(nullptr) > 0) {
    std::printf("FAIL device_bytes(null)\n");
    ++fails;
  }
  eosv_destroy(nullptr);
  // a long message through the thread-local error slot
  std::vector<int32_t> many(200, 1);
  expect_err(eosv_plan_episodes(many.data(), 200, 150, 1, 3, 2, nullptr, out, out), "plan: null outputs");
  std::printf(fails ? "asan_host args: %d failures\n" : "asan_host args: ok\n", fails);
  return fails ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && !std::strcmp(argv[1], "plan")) return plan(argc, argv);
  if (argc >= 2 && !std::strcmp(argv[1], "args")) return args();
  std::fprintf(stderr, "usage: asan_host plan N_WAY K_SHOT SEED N_EPISODES SIZE... | asan_host args\n");
  return 2;
}
