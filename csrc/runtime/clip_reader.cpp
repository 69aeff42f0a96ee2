// Native clip reader: parallel pread of selected frames of raw uint8 videos into a (pinned) host buffer.
//
// The reference decodes clips in 8 Python DataLoader worker processes per rank and ships fp32
// normalised clips.  Here the host side only has to move *raw* uint8 frames —
// and only the num_frames that UniformTemporalSubsample keeps — into pinned memory, from which one
// hipMemcpyAsync feeds the on-device preprocessing kernel.  The work runs on the thread pool of
// clip_reader_core.h with the GIL released.
#include <torch/extension.h>

#include "clip_reader_core.h"

namespace {

pva::ClipReader g_reader;
std::mutex g_reader_mu;

// jobs: list of (path, data_offset, frame_bytes, frame_indices, dst_offset)
void read_clips(const at::Tensor& dst, const std::vector<std::tuple<std::string, int64_t, int64_t,
                std::vector<int64_t>, int64_t>>& jobs, int64_t nthreads) {
  TORCH_CHECK(dst.scalar_type() == at::kByte && dst.is_contiguous() && !dst.is_cuda(), "dst: contiguous host uint8");
  std::vector<pva::ReadJob> rj;
  rj.reserve(jobs.size());
  for (const auto& j : jobs)
    rj.push_back({std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j), std::get<4>(j)});
  std::string err;
  {
    pybind11::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(g_reader_mu);
    err = g_reader.read(dst.data_ptr<uint8_t>(), dst.numel(), rj, (int)nthreads);
  }
  TORCH_CHECK(err.empty(), err);
}

}  // namespace

void register_clip_reader(pybind11::module& m) {
  m.def("read_clips", &read_clips, "parallel pread of raw uint8 frames into a host buffer",
        pybind11::arg("dst"), pybind11::arg("jobs"), pybind11::arg("nthreads") = 8);
}
