// Torch-free core of the native clip reader (csrc/runtime/clip_reader.cpp binds it to Python).
//
// A persistent std::thread pool executes one job per frame: pread(frame_bytes) at
// data_offset + index * frame_bytes into a caller-provided host (pinned) buffer.  File descriptors are
// cached per path.  Kept free of torch/pybind so tests/native/clip_reader_test.cpp can build it with
// -fsanitize=thread and -fsanitize=address,undefined (SURVEY.md §5 race detection / sanitizers).
#pragma once

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace pva {

class ThreadPool {
 public:
  explicit ThreadPool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  // Runs every job and returns when all have finished.  The completion count is decremented under the
  // waiter's mutex: a worker never touches the (stack-allocated) completion state after the waiter can
  // observe zero.
  void run_all(const std::vector<std::function<void()>>& jobs) {
    if (jobs.empty()) return;
    struct Done {
      std::mutex m;
      std::condition_variable cv;
      size_t left;
    } done;
    done.left = jobs.size();
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& j : jobs) {
        q_.push([&done, j] {
          j();
          std::lock_guard<std::mutex> g2(done.m);
          if (--done.left == 0) done.cv.notify_all();
        });
      }
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> l(done.m);
    done.cv.wait(l, [&] { return done.left == 0; });
  }
  size_t size() const { return workers_.size(); }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop();
      }
      f();
    }
  }
  std::vector<std::thread> workers_;
  std::queue<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct ReadJob {
  std::string path;
  int64_t data_offset;   // byte offset of frame 0 in the file
  int64_t frame_bytes;
  std::vector<int64_t> idx;  // frame indices to copy, in order
  int64_t dst_offset;    // byte offset in the destination buffer
};

class ClipReader {
 public:
  // Copies every job's frames into dst[0, cap).  Returns "" on success, else an error message.  Not
  // re-entrant: one call at a time per reader (the Python loader owns one reader per process).
  std::string read(uint8_t* dst, int64_t cap, const std::vector<ReadJob>& jobs, int nthreads) {
    nthreads = std::max(1, nthreads);
    if (fds_.size() > kMaxFds) close_all();  // evict only between calls: no queued job holds an fd
    std::vector<std::function<void()>> work;
    std::mutex emu;
    std::string err;
    for (const auto& j : jobs) {
      if (j.dst_offset < 0 || j.frame_bytes <= 0 ||
          j.dst_offset + (int64_t)j.idx.size() * j.frame_bytes > cap)
        return "clip reader destination overflow";
      const int fd = get_fd(j.path);
      if (fd < 0) return "cannot open " + j.path;
      for (size_t k = 0; k < j.idx.size(); ++k) {
        uint8_t* d = dst + j.dst_offset + (int64_t)k * j.frame_bytes;
        const int64_t src = j.data_offset + j.idx[k] * j.frame_bytes;
        const int64_t fb = j.frame_bytes;
        const std::string* path = &j.path;
        work.emplace_back([=, &emu, &err] {
          int64_t got = 0;
          while (got < fb) {
            const ssize_t r = ::pread(fd, d + got, fb - got, src + got);
            if (r <= 0) {
              std::lock_guard<std::mutex> g(emu);
              if (err.empty()) err = "short read from " + *path;
              return;
            }
            got += r;
          }
        });
      }
    }
    if (!pool_ || (int)pool_->size() != nthreads) pool_.reset(new ThreadPool(nthreads));
    pool_->run_all(work);
    return err;
  }
  ~ClipReader() {
    pool_.reset();
    close_all();
  }

 private:
  static constexpr size_t kMaxFds = 4096;
  int get_fd(const std::string& path) {
    auto it = fds_.find(path);
    if (it != fds_.end()) return it->second;
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd >= 0) fds_[path] = fd;
    return fd;
  }
  void close_all() {
    for (auto& kv : fds_) ::close(kv.second);
    fds_.clear();
  }
  std::unique_ptr<ThreadPool> pool_;
  std::unordered_map<std::string, int> fds_;
};

}  // namespace pva
