// Parameter-server sparse table: the server-side store behind paddle.distributed.ps (D13).
//
// Reference behaviour: paddle/fluid/distributed/ps/table/memory_sparse_table.{h,cc} (a sharded id -> value
// hash table created lazily on first pull, updated by pushes, with save / load / shrink), ctr_accessor.{h,cc}
// (per-feature show / click / unseen_days / delta_score statistics next to the embedding), sparse_sgd_rule.{h,cc}
// (naive SGD, AdaGrad with one g2sum per feature, Adam) and python/paddle/distributed/entry_attr.py (feature
// admission: count filter / probability).
//
// Layout: each shard owns a row arena (one contiguous float vector, `width` floats per feature, freed rows
// recycled) and an id -> row index. A row is [show, click, unseen_days, delta_score, seen, w[dim], state[..]].
// Pull / push group the ids by shard and process shards in parallel (std::thread) with the GIL released, so a
// server process serves several trainers' RPCs concurrently; each shard has its own mutex.
// Initial values are a pure function of (seed, id) (splitmix64), so they do not depend on arrival order.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline float u01(uint64_t h) { return static_cast<float>((h >> 40) * (1.0 / 16777216.0)); }

enum Rule { kSGD = 0, kAdaGrad = 1, kAdam = 2 };
enum Init { kUniform = 0, kNormal = 1, kZeros = 2 };
enum Entry { kNone = 0, kCountFilter = 1, kProbability = 2 };

// row header
constexpr int kShow = 0, kClick = 1, kUnseen = 2, kDelta = 3, kSeen = 4, kHead = 5;

class SparseTable {
 public:
  SparseTable(int dim, int rule, float lr, float init_range, int init, uint64_t seed, int entry, float entry_param,
              float initial_g2sum, float beta1, float beta2, float eps, float min_bound, float max_bound,
              int shard_num)
      : dim_(dim), rule_(rule), lr_(lr), init_range_(init_range), init_(init), seed_(seed), entry_(entry),
        entry_param_(entry_param), g2_init_(initial_g2sum), b1_(beta1), b2_(beta2), eps_(eps), lo_(min_bound),
        hi_(max_bound), shards_(std::max(shard_num, 1)) {
    if (dim <= 0) throw std::invalid_argument("SparseTable: dim must be > 0");
    state_ = rule == kSGD ? 0 : rule == kAdaGrad ? 1 : 2 * dim + 2;  // adam: m, v, beta1^t, beta2^t
    width_ = kHead + dim + state_;
  }

  int dim() const { return dim_; }

  // ids [n] -> out [n, dim]. training: create / admit missing features and reset unseen_days.
  void pull(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
            py::array_t<float, py::array::c_style> out, bool training) {
    const int64_t n = ids.size();
    if (out.size() != n * dim_) throw std::invalid_argument("pull: out must be [n, dim]");
    const int64_t* id = ids.data();
    float* o = out.mutable_data();
    py::gil_scoped_release nogil;
    for_shards(id, n, [&](Shard& s, const std::vector<int64_t>& idx) {
      std::lock_guard<std::mutex> g(s.mu);
      for (int64_t i : idx) {
        float* row = find(s, id[i], training);
        float* dst = o + i * dim_;
        if (row && admitted(row)) {
          if (training) row[kUnseen] = 0.f;
          std::memcpy(dst, row + kHead, sizeof(float) * dim_);
        } else {
          std::memset(dst, 0, sizeof(float) * dim_);
        }
      }
    });
  }

  // ids [n], grads [n, dim], optional shows / clicks [n]; unknown or not-yet-admitted features are skipped
  void push(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
            py::array_t<float, py::array::c_style | py::array::forcecast> grads, py::object shows,
            py::object clicks) {
    const int64_t n = ids.size();
    if (grads.size() != n * dim_) throw std::invalid_argument("push: grads must be [n, dim]");
    py::array_t<float, py::array::c_style | py::array::forcecast> sh, ck;
    const float* shp = nullptr;
    const float* ckp = nullptr;
    if (!shows.is_none()) {
      sh = shows.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      if (sh.size() != n) throw std::invalid_argument("push: shows must be [n]");
      shp = sh.data();
    }
    if (!clicks.is_none()) {
      ck = clicks.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      if (ck.size() != n) throw std::invalid_argument("push: clicks must be [n]");
      ckp = ck.data();
    }
    const int64_t* id = ids.data();
    const float* gr = grads.data();
    py::gil_scoped_release nogil;
    for_shards(id, n, [&](Shard& s, const std::vector<int64_t>& idx) {
      std::lock_guard<std::mutex> g(s.mu);
      for (int64_t i : idx) {
        float* row = find(s, id[i], false);
        if (!row) continue;
        row[kShow] += shp ? shp[i] : 1.f;
        row[kClick] += ckp ? ckp[i] : 0.f;
        if (!admitted(row)) continue;
        row[kDelta] += 1.f;
        update(row, gr + i * dim_);
      }
    });
  }

  int64_t size() const {
    int64_t t = 0;
    for (auto& s : shards_) t += static_cast<int64_t>(s.index.size());
    return t;
  }

  // decay statistics, age every feature by one pass, drop features unseen for more than `threshold` passes
  int64_t shrink(int64_t threshold, float decay) {
    py::gil_scoped_release nogil;
    int64_t dropped = 0;
    for (auto& s : shards_) {
      std::lock_guard<std::mutex> g(s.mu);
      for (auto it = s.index.begin(); it != s.index.end();) {
        float* row = s.rows.data() + static_cast<size_t>(it->second) * width_;
        row[kShow] *= decay;
        row[kClick] *= decay;
        row[kUnseen] += 1.f;
        if (row[kUnseen] > static_cast<float>(threshold)) {
          s.free.push_back(it->second);
          it = s.index.erase(it);
          ++dropped;
        } else {
          ++it;
        }
      }
    }
    return dropped;
  }

  // text format, one feature per line: id \t show \t click \t unseen \t w0,w1,... [\t state...]
  // mode 0: everything (with optimizer state); 1: delta (features updated since the last save), no state;
  // 2: base (weights only). After a save, delta scores are cleared.
  int64_t save(const std::string& path, int mode) {
    py::gil_scoped_release nogil;
    std::ofstream f(path);
    if (!f) throw std::runtime_error("SparseTable.save: cannot open " + path);
    int64_t count = 0;
    for (auto& s : shards_) {
      std::lock_guard<std::mutex> g(s.mu);
      for (auto& kv : s.index) {
        float* row = s.rows.data() + static_cast<size_t>(kv.second) * width_;
        if (mode == 1 && row[kDelta] <= 0.f) continue;
        f << kv.first << '\t' << row[kShow] << '\t' << row[kClick] << '\t' << row[kUnseen] << '\t' << row[kSeen]
          << '\t';
        write_vec(f, row + kHead, dim_);
        if (mode == 0 && state_ > 0) {
          f << '\t';
          write_vec(f, row + kHead + dim_, state_);
        }
        f << '\n';
        row[kDelta] = 0.f;
        ++count;
      }
    }
    return count;
  }

  int64_t load(const std::string& path) {
    py::gil_scoped_release nogil;
    std::ifstream f(path);
    if (!f) throw std::runtime_error("SparseTable.load: cannot open " + path);
    std::string line;
    int64_t count = 0;
    while (std::getline(f, line)) {
      if (line.empty()) continue;
      std::istringstream ls(line);
      std::string tok;
      std::vector<std::string> cols;
      while (std::getline(ls, tok, '\t')) cols.push_back(tok);
      if (cols.size() < 6) throw std::runtime_error("SparseTable.load: malformed line in " + path);
      const int64_t key = std::stoll(cols[0]);
      Shard& s = shards_[shard_of(key)];
      std::lock_guard<std::mutex> g(s.mu);
      float* row = create(s, key, /*init=*/false);
      row[kShow] = std::stof(cols[1]);
      row[kClick] = std::stof(cols[2]);
      row[kUnseen] = std::stof(cols[3]);
      row[kSeen] = std::stof(cols[4]);
      row[kDelta] = 0.f;
      read_vec(cols[5], row + kHead, dim_);
      if (cols.size() > 6 && state_ > 0) read_vec(cols[6], row + kHead + dim_, state_);
      else init_state(row);
      ++count;
    }
    return count;
  }

  // statistics of one feature (show, click, unseen_days, admitted) or None
  py::object stat(int64_t key) {
    Shard& s = shards_[shard_of(key)];
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.index.find(static_cast<uint64_t>(key));
    if (it == s.index.end()) return py::none();
    float* row = s.rows.data() + static_cast<size_t>(it->second) * width_;
    return py::make_tuple(row[kShow], row[kClick], row[kUnseen], admitted(row));
  }

  void set_lr(float lr) { lr_ = lr; }

 private:
  struct Shard {
    std::mutex mu;
    std::unordered_map<uint64_t, uint32_t> index;
    std::vector<float> rows;
    std::vector<uint32_t> free;
  };

  size_t shard_of(int64_t key) const { return splitmix64(static_cast<uint64_t>(key)) % shards_.size(); }

  template <class F>
  void for_shards(const int64_t* id, int64_t n, F&& fn) {
    const size_t S = shards_.size();
    std::vector<std::vector<int64_t>> parts(S);
    for (int64_t i = 0; i < n; ++i) parts[shard_of(id[i])].push_back(i);
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nthreads = n < 8192 ? 1 : std::min<size_t>({S, static_cast<size_t>(hw), 16});
    if (nthreads <= 1) {
      for (size_t k = 0; k < S; ++k)
        if (!parts[k].empty()) fn(shards_[k], parts[k]);
      return;
    }
    std::vector<std::thread> th;
    for (size_t t = 0; t < nthreads; ++t)
      th.emplace_back([&, t] {
        for (size_t k = t; k < S; k += nthreads)
          if (!parts[k].empty()) fn(shards_[k], parts[k]);
      });
    for (auto& x : th) x.join();
  }

  bool admitted(const float* row) const {
    if (entry_ == kCountFilter) return row[kShow] + 1e-6f >= entry_param_ || row[kSeen] > 0.5f;
    return row[kSeen] > 0.5f;
  }

  float* find(Shard& s, int64_t key, bool create_missing) {
    auto it = s.index.find(static_cast<uint64_t>(key));
    if (it != s.index.end()) {
      float* row = s.rows.data() + static_cast<size_t>(it->second) * width_;
      if (entry_ == kCountFilter && row[kSeen] < 0.5f && row[kShow] + 1e-6f >= entry_param_) {
        init_weights(row, key);  // admitted now: weights start from their initializer
        row[kSeen] = 1.f;
      }
      return row;
    }
    if (!create_missing) return nullptr;
    if (entry_ == kProbability) {
      // the admission draw is a function of the id: a rejected feature stays rejected for this seed
      if (u01(splitmix64(seed_ ^ (static_cast<uint64_t>(key) * 0xD6E8FEB86659FD93ull))) >= entry_param_)
        return nullptr;
    }
    return create(s, key, true);
  }

  float* create(Shard& s, int64_t key, bool init) {
    auto it = s.index.find(static_cast<uint64_t>(key));
    uint32_t slot;
    if (it != s.index.end()) {
      slot = it->second;
    } else if (!s.free.empty()) {
      slot = s.free.back();
      s.free.pop_back();
      s.index.emplace(static_cast<uint64_t>(key), slot);
    } else {
      slot = static_cast<uint32_t>(s.rows.size() / width_);
      s.rows.resize(s.rows.size() + width_);
      s.index.emplace(static_cast<uint64_t>(key), slot);
    }
    float* row = s.rows.data() + static_cast<size_t>(slot) * width_;
    std::fill(row, row + width_, 0.f);
    if (init) {
      const bool admit_now = entry_ != kCountFilter || entry_param_ <= 0.f;
      if (admit_now) {
        init_weights(row, key);
        row[kSeen] = 1.f;
      }
    }
    return row;
  }

  void init_weights(float* row, int64_t key) {
    float* w = row + kHead;
    for (int j = 0; j < dim_; ++j) {
      const uint64_t h = splitmix64(seed_ ^ splitmix64(static_cast<uint64_t>(key) * 1315423911ull + j));
      if (init_ == kZeros) {
        w[j] = 0.f;
      } else if (init_ == kUniform) {
        w[j] = (2.f * u01(h) - 1.f) * init_range_;
      } else {  // Box-Muller from two draws
        const float a = std::max(u01(h), 1e-7f), b = u01(splitmix64(h));
        w[j] = init_range_ * std::sqrt(-2.f * std::log(a)) * std::cos(6.2831853f * b);
      }
    }
    init_state(row);
  }

  void init_state(float* row) {
    float* st = row + kHead + dim_;
    std::fill(st, st + state_, 0.f);
    if (rule_ == kAdam) {
      st[2 * dim_] = b1_;
      st[2 * dim_ + 1] = b2_;
    }
  }

  float bound(float x) const { return std::min(std::max(x, lo_), hi_); }

  void update(float* row, const float* g) {
    float* w = row + kHead;
    float* st = w + dim_;
    if (rule_ == kSGD) {
      for (int j = 0; j < dim_; ++j) w[j] = bound(w[j] - lr_ * g[j]);
    } else if (rule_ == kAdaGrad) {
      // one accumulated squared-gradient per feature: w -= lr * g * sqrt(g2_0 / (g2_0 + g2sum))
      const float scale = std::sqrt(g2_init_ / (g2_init_ + st[0]));
      float add = 0.f;
      for (int j = 0; j < dim_; ++j) {
        w[j] = bound(w[j] - lr_ * g[j] * scale);
        add += g[j] * g[j];
      }
      st[0] += add / dim_;
    } else {
      float* m = st;
      float* v = st + dim_;
      float& b1p = st[2 * dim_];
      float& b2p = st[2 * dim_ + 1];
      const float lr_t = lr_ * std::sqrt(1.f - b2p) / (1.f - b1p);
      for (int j = 0; j < dim_; ++j) {
        m[j] = b1_ * m[j] + (1.f - b1_) * g[j];
        v[j] = b2_ * v[j] + (1.f - b2_) * g[j] * g[j];
        w[j] = bound(w[j] - lr_t * m[j] / (std::sqrt(v[j]) + eps_));
      }
      b1p *= b1_;
      b2p *= b2_;
    }
  }

  static void write_vec(std::ofstream& f, const float* v, int n) {
    char buf[32];
    for (int j = 0; j < n; ++j) {
      std::snprintf(buf, sizeof(buf), j ? ",%.9g" : "%.9g", v[j]);
      f << buf;
    }
  }

  static void read_vec(const std::string& s, float* v, int n) {
    const char* p = s.c_str();
    for (int j = 0; j < n; ++j) {
      char* end = nullptr;
      v[j] = std::strtof(p, &end);
      if (end == p) throw std::runtime_error("SparseTable.load: short vector");
      p = (*end == ',') ? end + 1 : end;
    }
  }

  int dim_, rule_;
  float lr_, init_range_;
  int init_;
  uint64_t seed_;
  int entry_;
  float entry_param_, g2_init_, b1_, b2_, eps_, lo_, hi_;
  int state_ = 0, width_ = 0;
  std::vector<Shard> shards_;
};

}  // namespace

void register_ps_table(py::module& m) {
  auto ps = m.def_submodule("ps", "parameter-server sparse table (MemorySparseTable equivalent)");
  py::class_<SparseTable>(ps, "SparseTable")
      .def(py::init<int, int, float, float, int, uint64_t, int, float, float, float, float, float, float, float,
                    int>(),
           py::arg("dim"), py::arg("rule") = 0, py::arg("lr") = 0.01f, py::arg("init_range") = 0.01f,
           py::arg("init") = 0, py::arg("seed") = 0, py::arg("entry") = 0, py::arg("entry_param") = 0.f,
           py::arg("initial_g2sum") = 3.f, py::arg("beta1") = 0.9f, py::arg("beta2") = 0.999f,
           py::arg("eps") = 1e-8f, py::arg("min_bound") = -1e30f, py::arg("max_bound") = 1e30f,
           py::arg("shard_num") = 16)
      .def("pull", &SparseTable::pull, py::arg("ids"), py::arg("out"), py::arg("training") = true)
      .def("push", &SparseTable::push, py::arg("ids"), py::arg("grads"), py::arg("shows") = py::none(),
           py::arg("clicks") = py::none())
      .def("size", &SparseTable::size)
      .def("dim", &SparseTable::dim)
      .def("shrink", &SparseTable::shrink, py::arg("threshold"), py::arg("decay") = 0.98f)
      .def("save", &SparseTable::save, py::arg("path"), py::arg("mode") = 0)
      .def("load", &SparseTable::load, py::arg("path"))
      .def("stat", &SparseTable::stat, py::arg("id"))
      .def("set_lr", &SparseTable::set_lr, py::arg("lr"));
}
