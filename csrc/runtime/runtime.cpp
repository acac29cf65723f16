// Native CPU-side runtime for paddlepaddle_amd (pybind11 module `_C_runtime`).
//
// Reference counterparts (C++ in the reference):
//   * batch assembly for the DataLoader       — paddle/fluid/operators/reader/, io/dataloader collate
//   * static-graph scheduling                 — paddle/fluid/framework/new_executor/program_interpreter.cc
//                                               (Build: dependency analysis, GC / last-use plan)
//   * gradient bucket planning                — paddle/fluid/distributed/collective/reducer.cc
//   * checkpoint tensor-file writer           — paddle/fluid/framework/io (SaveCombine)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <queue>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "allocator.h"

namespace py = pybind11;

namespace {

// Copy N equally-shaped contiguous arrays into out[N, ...] using a small thread team.
void stack_into(const std::vector<py::array>& arrs, py::array out) {
  const size_t n = arrs.size();
  if (n == 0) return;
  const size_t item = static_cast<size_t>(arrs[0].nbytes());
  if (static_cast<size_t>(out.nbytes()) != item * n) throw std::runtime_error("stack_into: size mismatch");
  std::vector<const char*> src(n);
  for (size_t i = 0; i < n; ++i) {
    if (static_cast<size_t>(arrs[i].nbytes()) != item) throw std::runtime_error("stack_into: ragged batch");
    src[i] = static_cast<const char*>(arrs[i].data());
  }
  char* dst = static_cast<char*>(out.mutable_data());
  const size_t total = item * n;
  unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency() / 2), 8u);
  if (total < (8u << 20)) nt = 1;  // small batches: threads cost more than the copy
  py::gil_scoped_release nogil;
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) std::memcpy(dst + i * item, src[i], item);
    return;
  }
  std::vector<std::thread> team;
  for (unsigned t = 0; t < nt; ++t) {
    team.emplace_back([&, t] {
      for (size_t i = t; i < n; i += nt) std::memcpy(dst + i * item, src[i], item);
    });
  }
  for (auto& th : team) th.join();
}

// Greedy bucketing in reverse registration order (≈ order in which grads become ready).
std::vector<std::vector<int64_t>> plan_buckets(const std::vector<int64_t>& sizes, int64_t bucket_bytes) {
  std::vector<std::vector<int64_t>> out;
  std::vector<int64_t> cur;
  int64_t acc = 0;
  for (int64_t i = static_cast<int64_t>(sizes.size()) - 1; i >= 0; --i) {
    cur.push_back(i);
    acc += sizes[i];
    if (acc >= bucket_bytes) {
      out.push_back(cur);
      cur.clear();
      acc = 0;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

// Kahn topological order (stable: among ready nodes the lowest priority class first, then the smallest id,
// i.e. program order when possible; the executor gives collectives class 0 so they are issued as soon as
// their inputs exist and overlap the independent compute) plus a last-use table: last[v] = position in
// `order` after which node v's output is dead.
py::tuple schedule(int64_t n, const std::vector<std::pair<int64_t, int64_t>>& edges, const std::vector<int64_t>& keep,
                   const std::vector<int64_t>& prio) {
  std::vector<std::vector<int64_t>> succ(n);
  std::vector<int64_t> indeg(n, 0);
  for (auto& e : edges) {
    if (e.first < 0 || e.first >= n || e.second < 0 || e.second >= n) throw std::runtime_error("schedule: bad edge");
    succ[e.first].push_back(e.second);
    indeg[e.second]++;
  }
  auto cls = [&](int64_t v) -> int64_t { return static_cast<int64_t>(prio.size()) == n ? prio[v] : 0; };
  using Item = std::pair<int64_t, int64_t>;  // (class, id)
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> ready;
  for (int64_t i = 0; i < n; ++i)
    if (indeg[i] == 0) ready.push({cls(i), i});
  std::vector<int64_t> order;
  order.reserve(n);
  while (!ready.empty()) {
    int64_t v = ready.top().second;
    ready.pop();
    order.push_back(v);
    for (int64_t w : succ[v])
      if (--indeg[w] == 0) ready.push({cls(w), w});
  }
  if (static_cast<int64_t>(order.size()) != n) throw std::runtime_error("schedule: graph has a cycle");
  std::vector<int64_t> pos(n);
  for (int64_t i = 0; i < n; ++i) pos[order[i]] = i;
  std::vector<char> kept(n, 0);
  for (int64_t k : keep)
    if (k >= 0 && k < n) kept[k] = 1;
  std::vector<int64_t> last(n, -1);
  for (int64_t v = 0; v < n; ++v) {
    if (kept[v]) continue;
    int64_t l = pos[v];
    for (int64_t w : succ[v]) l = std::max(l, pos[w]);
    last[v] = l;
  }
  return py::make_tuple(order, last);
}

// Dependency levels (ops in one level are independent -> candidates for separate HIP streams).
std::vector<int64_t> levels(int64_t n, const std::vector<std::pair<int64_t, int64_t>>& edges) {
  std::vector<std::vector<int64_t>> succ(n);
  std::vector<int64_t> indeg(n, 0), lvl(n, 0);
  for (auto& e : edges) {
    succ[e.first].push_back(e.second);
    indeg[e.second]++;
  }
  std::queue<int64_t> q;
  for (int64_t i = 0; i < n; ++i)
    if (!indeg[i]) q.push(i);
  while (!q.empty()) {
    int64_t v = q.front();
    q.pop();
    for (int64_t w : succ[v]) {
      lvl[w] = std::max(lvl[w], lvl[v] + 1);
      if (--indeg[w] == 0) q.push(w);
    }
  }
  return lvl;
}

// Raw tensor-file writer: header (JSON text written by Python) + concatenated 64-byte aligned blobs.
int64_t write_blobs(const std::string& path, const std::string& header, const std::vector<py::array>& blobs) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  uint64_t hl = header.size();
  f.write(reinterpret_cast<const char*>(&hl), 8);
  f.write(header.data(), static_cast<std::streamsize>(hl));
  int64_t off = 8 + static_cast<int64_t>(hl);
  static const char zeros[64] = {0};
  for (auto& b : blobs) {
    int64_t pad = (64 - off % 64) % 64;
    f.write(zeros, pad);
    off += pad;
    py::buffer_info info = b.request();
    const int64_t nb = static_cast<int64_t>(info.size * info.itemsize);
    {
      py::gil_scoped_release nogil;
      f.write(static_cast<const char*>(info.ptr), nb);
    }
    off += nb;
  }
  return off;
}

// Host-memory backend of the device allocator core (allocator.h) for CPU unit tests: "streams" are plain
// integers, cross-stream waits are counted.
void* host_raw_alloc(size_t n, int) { return std::aligned_alloc(4096, (n + 4095) / 4096 * 4096); }
void host_raw_free(void* p, int) { std::free(p); }
void host_wait(uintptr_t, uintptr_t, int) {}
void host_sync(int) {}

class HostAllocator {
 public:
  explicit HostAllocator(size_t min_chunk)
      : a_({host_raw_alloc, host_raw_free, host_wait, host_sync}, 0, min_chunk) {}
  uintptr_t allocate(size_t n, uintptr_t stream) { return reinterpret_cast<uintptr_t>(a_.allocate(n, stream)); }
  bool free(uintptr_t p) { return a_.deallocate(reinterpret_cast<void*>(p)); }
  size_t release() { return a_.release_free_chunks(); }
  size_t block_size(uintptr_t p) { return a_.block_size(reinterpret_cast<void*>(p)); }
  size_t free_blocks() { return a_.free_blocks(); }
  void begin_pool(uintptr_t stream, uint64_t pool) { a_.begin_pool(stream, pool); }
  void end_pool(uintptr_t stream) { a_.end_pool(stream); }
  void release_pool(uint64_t pool) { a_.release_pool(pool); }
  py::dict stats() {
    pa_alloc::Stats s = a_.stats();
    py::dict d;
    d["allocated"] = s.allocated; d["reserved"] = s.reserved; d["peak_allocated"] = s.peak_allocated;
    d["peak_reserved"] = s.peak_reserved; d["n_alloc"] = s.n_alloc; d["n_free"] = s.n_free;
    d["n_chunks"] = s.n_chunks; d["n_raw_alloc"] = s.n_raw_alloc; d["n_raw_free"] = s.n_raw_free;
    d["n_cross_stream"] = s.n_cross_stream; d["n_oom_release"] = s.n_oom_release;
    return d;
  }

 private:
  pa_alloc::BestFitAllocator a_;
};

}  // namespace

void register_pinned_pool(py::module& m);    // pinned_pool.cpp
void register_comm_watchdog(py::module& m);  // comm_watchdog.cpp
void register_ps_table(py::module& m);       // ps_table.cpp
void register_autograd_engine(py::module& m);  // autograd_engine.cpp

PYBIND11_MODULE(_C_runtime, m) {
  m.doc() = "paddlepaddle_amd native runtime (collate, scheduler, bucket planner, tensor files, pinned pool)";
  register_pinned_pool(m);
  register_comm_watchdog(m);
  register_ps_table(m);
  register_autograd_engine(m);
  py::class_<HostAllocator>(m, "HostAllocator")
      .def(py::init<size_t>(), py::arg("min_chunk") = size_t(64) << 20)
      .def("allocate", &HostAllocator::allocate, py::arg("nbytes"), py::arg("stream") = 0)
      .def("free", &HostAllocator::free)
      .def("release", &HostAllocator::release)
      .def("block_size", &HostAllocator::block_size)
      .def("free_blocks", &HostAllocator::free_blocks)
      .def("begin_pool", &HostAllocator::begin_pool)
      .def("end_pool", &HostAllocator::end_pool)
      .def("release_pool", &HostAllocator::release_pool)
      .def("stats", &HostAllocator::stats);
  m.def("stack_into", &stack_into, py::arg("arrays"), py::arg("out"));
  m.def("plan_buckets", &plan_buckets, py::arg("sizes"), py::arg("bucket_bytes"));
  m.def("schedule", &schedule, py::arg("n"), py::arg("edges"), py::arg("keep"),
        py::arg("prio") = std::vector<int64_t>());
  m.def("levels", &levels, py::arg("n"), py::arg("edges"));
  m.def("write_blobs", &write_blobs, py::arg("path"), py::arg("header"), py::arg("blobs"));
}
