// Native clip reader: parallel pread of selected frames of raw uint8 videos into a (pinned) host buffer.
//
// The reference decodes clips in 8 Python DataLoader worker processes per rank and ships fp32
// normalised clips.  Here the host side only has to move *raw* uint8 frames —
// and only the num_frames that UniformTemporalSubsample keeps — into pinned memory, from which one
// hipMemcpyAsync feeds the on-device preprocessing kernel.  A persistent std::thread pool executes
// one job per frame (pread of frame_bytes at data_offset + index * frame_bytes) with the GIL released;
// file descriptors are cached per path.
#include <torch/extension.h>

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  void run_all(std::vector<std::function<void()>>& jobs) {
    std::atomic<size_t> left(jobs.size());
    std::mutex dm;
    std::condition_variable dcv;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& j : jobs) {
        q_.push([&, j] {
          j();
          if (--left == 0) {
            std::lock_guard<std::mutex> g2(dm);
            dcv.notify_all();
          }
        });
      }
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> l(dm);
    dcv.wait(l, [&] { return left.load() == 0; });
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

std::unique_ptr<Pool> g_pool;
std::mutex g_fd_mu;
std::unordered_map<std::string, int> g_fds;

int get_fd(const std::string& path) {
  std::lock_guard<std::mutex> g(g_fd_mu);
  auto it = g_fds.find(path);
  if (it != g_fds.end()) return it->second;
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  TORCH_CHECK(fd >= 0, "cannot open ", path);
  if (g_fds.size() > 4096) {  // bound the cache
    for (auto& kv : g_fds) ::close(kv.second);
    g_fds.clear();
  }
  g_fds[path] = fd;
  return fd;
}

// jobs: list of (path, data_offset, frame_bytes, frame_indices, dst_offset)
void read_clips(const at::Tensor& dst, const std::vector<std::tuple<std::string, int64_t, int64_t,
                std::vector<int64_t>, int64_t>>& jobs, int64_t nthreads) {
  TORCH_CHECK(dst.scalar_type() == at::kByte && dst.is_contiguous() && !dst.is_cuda(), "dst: contiguous host uint8");
  uint8_t* base = dst.data_ptr<uint8_t>();
  const int64_t cap = dst.numel();
  std::vector<std::function<void()>> work;
  std::vector<std::string> errors;
  std::mutex emu;
  for (const auto& j : jobs) {
    const std::string& path = std::get<0>(j);
    const int64_t off0 = std::get<1>(j), fb = std::get<2>(j), dsto = std::get<4>(j);
    const auto& idx = std::get<3>(j);
    TORCH_CHECK(dsto + (int64_t)idx.size() * fb <= cap, "clip reader destination overflow");
    const int fd = get_fd(path);
    for (size_t k = 0; k < idx.size(); ++k) {
      uint8_t* d = base + dsto + (int64_t)k * fb;
      const int64_t src = off0 + idx[k] * fb;
      work.emplace_back([=, &errors, &emu] {
        int64_t done = 0;
        while (done < fb) {
          ssize_t r = ::pread(fd, d + done, fb - done, src + done);
          if (r <= 0) {
            std::lock_guard<std::mutex> g(emu);
            errors.push_back(path);
            return;
          }
          done += r;
        }
      });
    }
  }
  {
    pybind11::gil_scoped_release nogil;
    if (!g_pool || (int64_t)g_pool->size() != nthreads) g_pool.reset(new Pool((int)std::max<int64_t>(1, nthreads)));
    g_pool->run_all(work);
  }
  TORCH_CHECK(errors.empty(), "short read from ", errors.empty() ? "" : errors[0]);
}

}  // namespace

void register_clip_reader(pybind11::module& m) {
  m.def("read_clips", &read_clips, "parallel pread of raw uint8 frames into a host buffer",
        pybind11::arg("dst"), pybind11::arg("jobs"), pybind11::arg("nthreads") = 8);
}
