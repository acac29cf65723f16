// Collective-communication watchdog: failure / hang detection for RCCL collectives.
//
// Reference behaviour: paddle/phi/core/distributed/comm_task_manager.cc (CommTaskManager: a background
// thread that walks the outstanding comm tasks, checks their CUDA events, and reports — and optionally
// aborts — tasks that exceed the timeout, with op / rank / group / size details) and comm_task.h.
//
// Here every tracked collective gets a HIP event recorded on the stream that consumes its result, right
// after the collective is issued. A native thread polls the events (hipEventQuery, resolved at run time
// from the HIP runtime torch already loaded, like the pinned pool) every `poll_ms`; completed tasks are
// retired (event destroyed), a task still pending after `timeout_ms` is reported once on stderr and in a
// per-rank report file (`<dir>/comm_watchdog.rank<r>.txt`) together with every other pending task, and
// the process is aborted if `abort_on_timeout` is set (the reference's FLAGS_... abort path). Host-side
// tasks (gloo / CPU) are tracked by explicit `finish(id)` calls instead of events.
#include <dlfcn.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

using EventCreateFn = int (*)(void**, unsigned);
using EventRecordFn = int (*)(void*, void*);
using EventQueryFn = int (*)(void*);
using EventDestroyFn = int (*)(void*);

struct HipEvents {
  EventCreateFn create = nullptr;
  EventRecordFn record = nullptr;
  EventQueryFn query = nullptr;
  EventDestroyFn destroy = nullptr;
  bool ok() const { return create && record && query && destroy; }
};

HipEvents resolve_events() {
  HipEvents h;
  const char* names[] = {"libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"};
  for (const char* n : names) {
    void* lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (!lib) continue;
    h.create = reinterpret_cast<EventCreateFn>(dlsym(lib, "hipEventCreateWithFlags"));
    h.record = reinterpret_cast<EventRecordFn>(dlsym(lib, "hipEventRecord"));
    h.query = reinterpret_cast<EventQueryFn>(dlsym(lib, "hipEventQuery"));
    h.destroy = reinterpret_cast<EventDestroyFn>(dlsym(lib, "hipEventDestroy"));
    if (h.ok()) break;
  }
  return h;
}

constexpr int kHipSuccess = 0;
constexpr unsigned kHipEventDisableTiming = 0x2;

struct Task {
  std::string op, group;
  int64_t bytes = 0;
  void* event = nullptr;  // nullptr: host task, finished explicitly
  std::chrono::steady_clock::time_point start;
  int64_t timeout_ms = 0;
  bool reported = false;
};

class Watchdog {
 public:
  static Watchdog& get() {
    static Watchdog w;
    return w;
  }

  void start(int rank, int64_t timeout_ms, int64_t poll_ms, bool abort_on_timeout, const std::string& report_dir) {
    std::lock_guard<std::mutex> g(mu_);
    rank_ = rank;
    default_timeout_ms_ = timeout_ms;
    poll_ms_ = poll_ms;
    abort_ = abort_on_timeout;
    dir_ = report_dir;
    if (!hip_.ok()) hip_ = resolve_events();
    if (!running_) {
      running_ = true;
      th_ = std::thread([this] { loop(); });
    }
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!running_) return;
      running_ = false;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : tasks_)
      if (kv.second.event && hip_.ok()) hip_.destroy(kv.second.event);
    tasks_.clear();
  }

  // device task: an event is recorded on `stream` (hipStream_t as integer; 0 = null stream)
  int64_t track(const std::string& op, const std::string& group, int64_t bytes, uintptr_t stream,
                int64_t timeout_ms) {
    Task t;
    t.op = op;
    t.group = group;
    t.bytes = bytes;
    t.start = std::chrono::steady_clock::now();
    t.timeout_ms = timeout_ms > 0 ? timeout_ms : default_timeout_ms_;
    if (hip_.ok()) {
      void* ev = nullptr;
      if (hip_.create(&ev, kHipEventDisableTiming) == kHipSuccess) {
        if (hip_.record(ev, reinterpret_cast<void*>(stream)) == kHipSuccess) t.event = ev;
        else hip_.destroy(ev);
      }
    }
    std::lock_guard<std::mutex> g(mu_);
    const int64_t id = next_id_++;
    tasks_.emplace(id, std::move(t));
    return id;
  }

  int64_t track_host(const std::string& op, const std::string& group, int64_t bytes, int64_t timeout_ms) {
    Task t;
    t.op = op;
    t.group = group;
    t.bytes = bytes;
    t.start = std::chrono::steady_clock::now();
    t.timeout_ms = timeout_ms > 0 ? timeout_ms : default_timeout_ms_;
    std::lock_guard<std::mutex> g(mu_);
    const int64_t id = next_id_++;
    tasks_.emplace(id, std::move(t));
    return id;
  }

  void finish(int64_t id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tasks_.find(id);
    if (it == tasks_.end()) return;
    if (it->second.event && hip_.ok()) hip_.destroy(it->second.event);
    tasks_.erase(it);
  }

  int64_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return static_cast<int64_t>(tasks_.size());
  }

  int64_t timeouts() const { return n_timeouts_.load(); }

  std::vector<std::string> timed_out_ops() {
    std::lock_guard<std::mutex> g(mu_);
    return timed_out_;
  }

  bool device_events() const { return hip_.ok(); }

 private:
  Watchdog() = default;
  ~Watchdog() {
    // process exit: do not join (the HIP runtime may already be torn down); just stop polling
    running_ = false;
    cv_.notify_all();
    if (th_.joinable()) th_.detach();
  }

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (running_) {
      cv_.wait_for(lk, std::chrono::milliseconds(poll_ms_));
      if (!running_) break;
      const auto now = std::chrono::steady_clock::now();
      std::vector<int64_t> done;
      bool fire = false;
      for (auto& kv : tasks_) {
        Task& t = kv.second;
        if (t.event && hip_.query(t.event) == kHipSuccess) {
          done.push_back(kv.first);
          continue;
        }
        const int64_t age = std::chrono::duration_cast<std::chrono::milliseconds>(now - t.start).count();
        if (!t.reported && age > t.timeout_ms) {
          t.reported = true;
          fire = true;
          n_timeouts_++;
          timed_out_.push_back(t.op);
        }
      }
      for (int64_t id : done) {
        auto it = tasks_.find(id);
        if (it->second.event) hip_.destroy(it->second.event);
        tasks_.erase(it);
      }
      if (fire) report(now);
      if (fire && abort_) {
        std::fflush(stderr);
        std::abort();
      }
    }
  }

  void report(std::chrono::steady_clock::time_point now) {
    std::string msg = "[comm_watchdog] rank " + std::to_string(rank_) + ": collective(s) exceeded their timeout; pending:\n";
    for (auto& kv : tasks_) {
      const Task& t = kv.second;
      const int64_t age = std::chrono::duration_cast<std::chrono::milliseconds>(now - t.start).count();
      msg += "  task " + std::to_string(kv.first) + " op=" + t.op + " group=" + t.group + " bytes=" +
             std::to_string(t.bytes) + " age_ms=" + std::to_string(age) + " timeout_ms=" +
             std::to_string(t.timeout_ms) + (t.event ? " (device)" : " (host)") + "\n";
    }
    std::fputs(msg.c_str(), stderr);
    if (!dir_.empty()) {
      std::ofstream f(dir_ + "/comm_watchdog.rank" + std::to_string(rank_) + ".txt", std::ios::app);
      f << msg;
    }
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  bool running_ = false;
  HipEvents hip_;
  std::map<int64_t, Task> tasks_;
  int64_t next_id_ = 1;
  int rank_ = 0;
  int64_t default_timeout_ms_ = 600000;
  int64_t poll_ms_ = 1000;
  bool abort_ = false;
  std::string dir_;
  std::atomic<int64_t> n_timeouts_{0};
  std::vector<std::string> timed_out_;
};

}  // namespace

void register_comm_watchdog(py::module& m) {
  auto w = m.def_submodule("comm_watchdog", "native collective watchdog (CommTaskManager equivalent)");
  w.def("start", [](int rank, int64_t timeout_ms, int64_t poll_ms, bool abort_on_timeout, const std::string& dir) {
          Watchdog::get().start(rank, timeout_ms, poll_ms, abort_on_timeout, dir);
        },
        py::arg("rank"), py::arg("timeout_ms"), py::arg("poll_ms"), py::arg("abort_on_timeout"), py::arg("report_dir"));
  w.def("stop", [] {
    py::gil_scoped_release nogil;
    Watchdog::get().stop();
  });
  w.def("track", [](const std::string& op, const std::string& group, int64_t bytes, uintptr_t stream,
                    int64_t timeout_ms) { return Watchdog::get().track(op, group, bytes, stream, timeout_ms); },
        py::arg("op"), py::arg("group"), py::arg("bytes"), py::arg("stream"), py::arg("timeout_ms") = 0);
  w.def("track_host", [](const std::string& op, const std::string& group, int64_t bytes, int64_t timeout_ms) {
          return Watchdog::get().track_host(op, group, bytes, timeout_ms);
        },
        py::arg("op"), py::arg("group"), py::arg("bytes"), py::arg("timeout_ms") = 0);
  w.def("finish", [](int64_t id) { Watchdog::get().finish(id); });
  w.def("pending", [] { return Watchdog::get().pending(); });
  w.def("timeouts", [] { return Watchdog::get().timeouts(); });
  w.def("timed_out_ops", [] { return Watchdog::get().timed_out_ops(); });
  w.def("device_events", [] { return Watchdog::get().device_events(); });
}
