// KITTI .bin point-cloud streaming into device memory.
//
// Reference: data_process/kitti_dataset.py:119-122 get_lidar =
//   np.fromfile(path, dtype=np.float32).reshape(-1, 4)
// (a file whose float count is not a multiple of 4 makes reshape raise; trailing bytes
// that do not form a whole float are ignored by fromfile).
//
// The reference reads one file per DataLoader item and voxelises it on the CPU (≈40
// frames/s/core).  Here a producer thread reads whole batches of files with a pool of
// pread() workers into one of two host staging slots (pinned with hipHostMalloc, so the
// H2D copy is a DMA that overlaps the GPU work of the previous batch); next() hands a
// ready slot to the caller's stream with hipMemcpyAsync and records an event, and the
// producer refills the slot only after that event has completed.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace {

struct Slot {
  float* host = nullptr;
  int64_t cap_points = 0;
  std::vector<int64_t> offs;  // batch + 1
  int nframes = 0;
  enum State { FREE, FILLING, READY, IN_FLIGHT } state = FREE;
  int rc = SFA_OK;
  std::string err;
  hipEvent_t done = nullptr;
};

}  // namespace

struct sfa_bin_stream {
  std::vector<std::string> paths;
  int batch = 0, nthreads = 1;
  bool pinned = true;
  Slot slot[2];
  int next_fill = 0;     // next batch index the producer reads
  int next_take = 0;     // next batch index next() returns
  int nbatches = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool stop = false;
  // sticky failure: once a hand-off to the device failed, every later next() returns it
  // (the slot's state is unknown, so no batch is ever handed out from it again)
  int failed = SFA_OK;
  std::string failed_err;
  std::thread producer;
};

namespace {

// np.fromfile(path, float32).reshape(-1, 4) semantics; returns points or -1 (error set)
int64_t file_points(const std::string& p, std::string& err) {
  struct stat st;
  if (stat(p.c_str(), &st) != 0) {
    err = "cannot stat " + p;
    return -1;
  }
  const int64_t nfloat = (int64_t)st.st_size / 4;
  if (nfloat % 4 != 0) {
    err = p + ": float count not a multiple of 4 (reshape(-1, 4) would raise)";
    return -1;
  }
  return nfloat / 4;
}

int read_exact(const std::string& p, char* dst, int64_t bytes, std::string& err) {
  const int fd = open(p.c_str(), O_RDONLY);
  if (fd < 0) {
    err = "cannot open " + p;
    return -1;
  }
  int64_t got = 0;
  while (got < bytes) {
    const ssize_t r = pread(fd, dst + got, (size_t)(bytes - got), (off_t)got);
    if (r <= 0) {
      close(fd);
      err = "short read on " + p;
      return -1;
    }
    got += r;
  }
  close(fd);
  return 0;
}

void fill_slot(sfa_bin_stream* s, Slot& sl, int b) {
  const int f0 = b * s->batch;
  const int n = std::min(s->batch, (int)s->paths.size() - f0);
  sl.nframes = n;
  sl.rc = SFA_OK;
  sl.err.clear();
  sl.offs.assign(s->batch + 1, 0);
  for (int i = 0; i < n; ++i) {
    const int64_t np_ = file_points(s->paths[f0 + i], sl.err);
    if (np_ < 0) {
      sl.rc = SFA_E_INVALID;
      return;
    }
    sl.offs[i + 1] = sl.offs[i] + np_;
  }
  for (int i = n; i < s->batch; ++i) sl.offs[i + 1] = sl.offs[n];
  if (sl.offs[n] > sl.cap_points) {
    sl.rc = SFA_E_WORKSPACE;
    sl.err = "batch " + std::to_string(b) + " has " + std::to_string(sl.offs[n]) +
             " points > max_points_per_batch " + std::to_string(sl.cap_points);
    return;
  }
  // files dealt round-robin to the readers
  std::vector<std::thread> pool;
  std::vector<std::string> errs(s->nthreads);
  std::atomic<int> bad{0};
  const int nt = std::max(1, std::min(s->nthreads, n));
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&, t] {
      for (int i = t; i < n; i += nt)
        if (read_exact(s->paths[f0 + i], reinterpret_cast<char*>(sl.host + 4 * sl.offs[i]),
                       (sl.offs[i + 1] - sl.offs[i]) * 16, errs[t]) != 0)
          bad.fetch_add(1);
    });
  for (auto& th : pool) th.join();
  if (bad.load()) {
    sl.rc = SFA_E_INVALID;
    for (auto& e : errs)
      if (!e.empty()) sl.err = e;
  }
}

void producer_loop(sfa_bin_stream* s) {
  for (;;) {
    Slot* sl;
    int b;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv.wait(lk, [&] {
        return s->stop || (s->next_fill < s->nbatches &&
                           (s->slot[s->next_fill & 1].state == Slot::FREE ||
                            s->slot[s->next_fill & 1].state == Slot::IN_FLIGHT));
      });
      if (s->stop || s->next_fill >= s->nbatches) return;
      b = s->next_fill++;
      sl = &s->slot[b & 1];
      if (sl->state == Slot::IN_FLIGHT) {
        // the previous batch in this slot is still being copied to the device
        lk.unlock();
        if (sl->done) (void)hipEventSynchronize(sl->done);
        lk.lock();
      }
      sl->state = Slot::FILLING;
    }
    fill_slot(s, *sl, b);
    {
      std::lock_guard<std::mutex> lk(s->mu);
      sl->state = Slot::READY;
    }
    s->cv.notify_all();
  }
}

}  // namespace

using namespace sfa;

extern "C" int sfa_bin_stream_create(const char* const* paths, int n_files, int batch,
                                     int64_t max_points_per_batch, int n_threads, int pinned,
                                     sfa_bin_stream** out) {
  SFA_CHECK_ARG(out && (n_files == 0 || paths) && n_files >= 0 && batch >= 1 &&
                    max_points_per_batch >= 1 && n_threads >= 1,
                "bin_stream: bad arguments");
  auto* s = new sfa_bin_stream;
  for (int i = 0; i < n_files; ++i) {
    if (!paths[i]) {
      delete s;
      set_error("bin_stream: null path %d", i);
      return SFA_E_INVALID;
    }
    s->paths.emplace_back(paths[i]);
  }
  s->batch = batch;
  s->nthreads = n_threads;
  s->pinned = pinned != 0;
  s->nbatches = (n_files + batch - 1) / batch;
  for (auto& sl : s->slot) {
    sl.cap_points = max_points_per_batch;
    const size_t bytes = (size_t)max_points_per_batch * 16;
    if (s->pinned) {
      if (hipHostMalloc(reinterpret_cast<void**>(&sl.host), bytes, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
        sfa_bin_stream_destroy(s);
        set_error("bin_stream: pinned host allocation of %zu bytes failed", bytes);
        return SFA_E_HIP;
      }
    } else {
      sl.host = static_cast<float*>(malloc(bytes));
      if (!sl.host) {
        sfa_bin_stream_destroy(s);
        set_error("bin_stream: host allocation of %zu bytes failed", bytes);
        return SFA_E_INVALID;
      }
    }
  }
  s->producer = std::thread(producer_loop, s);
  *out = s;
  return SFA_OK;
}

extern "C" int sfa_bin_stream_next(sfa_bin_stream* s, float* points, int64_t capacity_points,
                                   int64_t* frame_offsets, int* n_frames, void* stream) {
  SFA_CHECK_ARG(s && points && frame_offsets && n_frames, "bin_stream_next: null argument");
  std::unique_lock<std::mutex> lk(s->mu);
  if (s->failed != SFA_OK) {
    set_error("%s", s->failed_err.c_str());
    return s->failed;
  }
  if (s->next_take >= s->nbatches) {
    *n_frames = 0;
    for (int i = 0; i <= s->batch; ++i) frame_offsets[i] = 0;
    return SFA_OK;
  }
  Slot& sl = s->slot[s->next_take & 1];
  s->cv.wait(lk, [&] { return sl.state == Slot::READY; });
  const int b = s->next_take++;
  if (sl.rc != SFA_OK) {
    sl.state = Slot::FREE;
    lk.unlock();
    s->cv.notify_all();
    set_error("bin_stream: batch %d: %s", b, sl.err.c_str());
    return sl.rc;
  }
  const int64_t npts = sl.offs[sl.nframes];
  if (npts > capacity_points) {
    sl.state = Slot::FREE;
    lk.unlock();
    s->cv.notify_all();
    set_error("bin_stream: batch %d has %lld points > capacity %lld", b, (long long)npts,
              (long long)capacity_points);
    return SFA_E_WORKSPACE;
  }
  for (int i = 0; i <= s->batch; ++i) frame_offsets[i] = sl.offs[i];
  *n_frames = sl.nframes;
  if (s->pinned) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipError_t e = npts > 0 ? hipMemcpyAsync(points, sl.host, (size_t)npts * 16, hipMemcpyHostToDevice, st)
                            : hipSuccess;
    const bool copied = e == hipSuccess && npts > 0;
    if (e == hipSuccess) e = hipEventRecord(sl.done, st);
    if (e != hipSuccess) {
      // the copy may be in flight with no event to wait on: drain the stream (best effort)
      // before anyone may touch the slot, stop the producer and fail every later call
      if (copied) (void)hipStreamSynchronize(st);
      s->failed = SFA_E_HIP;
      s->failed_err = std::string("bin_stream: batch ") + std::to_string(b) + ": device hand-off failed: " +
                      hipGetErrorString(e);
      s->stop = true;
      sl.state = Slot::FREE;
      lk.unlock();
      s->cv.notify_all();
      set_error("%s", s->failed_err.c_str());
      return SFA_E_HIP;
    }
    sl.state = Slot::IN_FLIGHT;  // the producer waits for `done` before refilling
  } else {
    memcpy(points, sl.host, (size_t)npts * 16);  // host destination (no device involved)
    sl.state = Slot::FREE;
  }
  lk.unlock();
  s->cv.notify_all();
  return SFA_OK;
}

extern "C" void sfa_bin_stream_destroy(sfa_bin_stream* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->stop = true;
  }
  s->cv.notify_all();
  if (s->producer.joinable()) s->producer.join();
  for (auto& sl : s->slot) {
    if (sl.done) {
      (void)hipEventSynchronize(sl.done);
      (void)hipEventDestroy(sl.done);
    }
    if (sl.host) {
      if (s->pinned)
        (void)hipHostFree(sl.host);
      else
        free(sl.host);
    }
  }
  delete s;
}
