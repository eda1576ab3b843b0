// Host-sanitizer driver for csrc/binstream.cpp (host ASan/UBSan/TSan are this
// build's race-detection counterpart).  Built by tests/test_binstream.py twice — with
// -fsanitize=address,undefined and with -fsanitize=thread — against binstream.cpp itself, and
// run in host mode (pinned = 0: no HIP call is made, so no GPU is needed).
//
// It exercises the producer thread + pread pool + two-slot state machine:
//   * every batch equals the files' bytes (np.fromfile(...).reshape(-1, 4), kitti_dataset.py:119-122),
//     for several batch sizes / reader counts, ragged and empty files, a short last batch;
//   * the consumer racing the producer (no sleeps: the slots hand over as fast as they can);
//   * destroy while the producer is mid-batch or blocked on a full slot (early exit);
//   * error batches (a file whose float count is not a multiple of 4, a missing file, a batch
//     over capacity) followed by further next() calls.
// Exit code 0 = every check passed (a sanitizer report aborts with a non-zero code).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sfa_hip.h"

namespace sfa {
// the library's error sink lives in model.hip; the driver links binstream.cpp alone
static std::string g_last;
void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last = buf;
}
}  // namespace sfa

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
      ++fails;                                                    \
    }                                                             \
  } while (0)

static std::vector<float> write_file(const std::string& path, int64_t npts, unsigned seed, int extra_bytes = 0) {
  std::vector<float> v((size_t)npts * 4);
  unsigned x = seed * 2654435761u + 1;
  for (auto& f : v) {
    x = x * 1664525u + 1013904223u;
    f = (float)(x >> 8) / 16777216.0f - 0.5f;
  }
  FILE* fp = fopen(path.c_str(), "wb");
  if (!fp) {
    perror(path.c_str());
    exit(2);
  }
  if (!v.empty()) fwrite(v.data(), 4, v.size(), fp);
  for (int i = 0; i < extra_bytes; ++i) fputc(0, fp);
  fclose(fp);
  return v;
}

static void stream_all(const std::vector<std::string>& paths, const std::vector<std::vector<float>>& data,
                       int batch, int threads, int64_t cap) {
  std::vector<const char*> cp;
  for (auto& p : paths) cp.push_back(p.c_str());
  sfa_bin_stream* s = nullptr;
  CHECK(sfa_bin_stream_create(cp.data(), (int)cp.size(), batch, cap, threads, 0, &s) == SFA_OK);
  std::vector<float> pts((size_t)cap * 4);
  std::vector<int64_t> offs(batch + 1);
  size_t file = 0;
  for (;;) {
    int n = -1;
    CHECK(sfa_bin_stream_next(s, pts.data(), cap, offs.data(), &n, nullptr) == SFA_OK);
    if (n <= 0) break;
    for (int i = 0; i < n; ++i, ++file) {
      const auto& d = data[file];
      CHECK((size_t)(offs[i + 1] - offs[i]) * 4 == d.size());
      CHECK(d.empty() || memcmp(pts.data() + 4 * offs[i], d.data(), d.size() * 4) == 0);
    }
  }
  CHECK(file == paths.size());
  sfa_bin_stream_destroy(s);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const int64_t sizes[] = {1000, 0, 131072, 7, 50000, 1, 99999, 123457, 5, 60000, 3, 4096, 17};
  std::vector<std::string> paths;
  std::vector<std::vector<float>> data;
  int64_t total = 0;
  for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; ++i) {
    paths.push_back(dir + "/f" + std::to_string(i) + ".bin");
    data.push_back(write_file(paths.back(), sizes[i], (unsigned)i, i == 3 ? 2 : 0));  // 2 trailing bytes
    total += sizes[i];
  }
  for (int batch : {1, 2, 3, 4, 16})
    for (int threads : {1, 3, 8})
      for (int rep = 0; rep < 3; ++rep) stream_all(paths, data, batch, threads, total);

  // early destroy: the producer is reading / waiting on a full slot
  {
    std::vector<const char*> cp;
    for (auto& p : paths) cp.push_back(p.c_str());
    for (int taken = 0; taken < 4; ++taken) {
      sfa_bin_stream* s = nullptr;
      CHECK(sfa_bin_stream_create(cp.data(), (int)cp.size(), 2, total, 4, 0, &s) == SFA_OK);
      std::vector<float> pts((size_t)total * 4);
      std::vector<int64_t> offs(3);
      for (int k = 0; k < taken; ++k) {
        int n = 0;
        CHECK(sfa_bin_stream_next(s, pts.data(), total, offs.data(), &n, nullptr) == SFA_OK);
      }
      sfa_bin_stream_destroy(s);
    }
  }

  // error batches, then the stream keeps going (host mode: a bad batch is skipped)
  {
    const std::string bad = dir + "/bad.bin";
    write_file(bad, 3, 99, 4);  // 13 floats: reshape(-1, 4) would raise
    const std::string missing = dir + "/missing.bin";
    std::vector<std::string> ps = {paths[0], bad, paths[2], missing, paths[4], paths[5]};
    std::vector<const char*> cp;
    for (auto& p : ps) cp.push_back(p.c_str());
    sfa_bin_stream* s = nullptr;
    CHECK(sfa_bin_stream_create(cp.data(), (int)cp.size(), 1, 200000, 2, 0, &s) == SFA_OK);
    std::vector<float> pts(200000 * 4);
    std::vector<int64_t> offs(2);
    int rcs[7];
    for (int k = 0; k < 7; ++k) {
      int n = 0;
      rcs[k] = sfa_bin_stream_next(s, pts.data(), 200000, offs.data(), &n, nullptr);
    }
    CHECK(rcs[0] == SFA_OK && rcs[1] == SFA_E_INVALID && rcs[2] == SFA_OK && rcs[3] == SFA_E_INVALID &&
          rcs[4] == SFA_OK && rcs[5] == SFA_OK && rcs[6] == SFA_OK);
    sfa_bin_stream_destroy(s);
    // over capacity: the slot's own cap, then the caller's
    const char* two[] = {paths[2].c_str(), paths[7].c_str()};
    CHECK(sfa_bin_stream_create(two, 2, 2, 1000, 2, 0, &s) == SFA_OK);
    int n = 0;
    CHECK(sfa_bin_stream_next(s, pts.data(), 1000, offs.data(), &n, nullptr) == SFA_E_WORKSPACE);
    sfa_bin_stream_destroy(s);
    CHECK(sfa_bin_stream_create(two, 2, 1, 200000, 2, 0, &s) == SFA_OK);
    CHECK(sfa_bin_stream_next(s, pts.data(), 10, offs.data(), &n, nullptr) == SFA_E_WORKSPACE);
    CHECK(sfa_bin_stream_next(s, pts.data(), 200000, offs.data(), &n, nullptr) == SFA_OK && n == 1);
    sfa_bin_stream_destroy(s);
  }
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("binstream sanitize ok\n");
  return 0;
}
