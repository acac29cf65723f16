// Auto-growth best-fit pool of page-locked (pinned) host memory.
//
// Reference behaviour: paddle/phi/core/memory/allocation/auto_growth_best_fit_allocator.cc (chunked
// growth, best-fit free blocks, split + coalesce) over pinned_allocator.cc (cudaHostAlloc). Here the
// chunks come from hipHostMalloc, resolved at run time from the HIP runtime that torch already loaded
// (dlopen RTLD_NOLOAD), so this CPU runtime library has no link-time HIP dependency; on a host without
// a HIP device the pool falls back to page-aligned pageable memory and reports ``pinned = false``.
//
// Pinned buffers feed asynchronous host->device copies (DataLoader pin_memory, Tensor.pin_memory,
// checkpoint staging). Stream safety (do not reuse a block while a copy still reads it) is handled by
// the Python owner, which defers the free until the copy's event completes.
#include <dlfcn.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

using HostMallocFn = int (*)(void**, size_t, unsigned);
using HostFreeFn = int (*)(void*);

struct HipHost {
  HostMallocFn alloc = nullptr;
  HostFreeFn release = nullptr;
};

HipHost resolve_hip() {
  HipHost h;
  const char* names[] = {"libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"};
  for (const char* n : names) {
    void* lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (!lib) continue;
    h.alloc = reinterpret_cast<HostMallocFn>(dlsym(lib, "hipHostMalloc"));
    h.release = reinterpret_cast<HostFreeFn>(dlsym(lib, "hipHostFree"));
    if (h.alloc && h.release) return h;
  }
  return HipHost{};
}

class PinnedPool {
 public:
  PinnedPool(size_t chunk_bytes, size_t alignment, bool use_hip)
      : chunk_bytes_(chunk_bytes), align_(alignment ? alignment : 256) {
    if (use_hip) hip_ = resolve_hip();
  }
  ~PinnedPool() {
    for (Chunk* c : chunks_) free_chunk(c);
  }

  bool pinned() const { return hip_.alloc != nullptr; }

  uintptr_t allocate(size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    const size_t need = round_up(n ? n : 1);
    auto it = free_.lower_bound(need);  // best fit: smallest free block that holds the request
    Block* b = nullptr;
    if (it != free_.end()) {
      b = it->second;
      free_.erase(it);
      ++hits_;
    } else {
      b = grow(need);
      if (!b) throw std::bad_alloc();
    }
    split(b, need);
    b->free = false;
    live_[b->ptr] = b;
    allocated_ += b->size;
    if (allocated_ > peak_) peak_ = allocated_;
    ++n_alloc_;
    return reinterpret_cast<uintptr_t>(b->ptr);
  }

  void deallocate(uintptr_t p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(reinterpret_cast<char*>(p));
    if (it == live_.end()) throw std::invalid_argument("PinnedPool: pointer not owned by this pool");
    Block* b = it->second;
    live_.erase(it);
    allocated_ -= b->size;
    b->free = true;
    // coalesce with free neighbours of the same chunk (address-ordered list)
    if (b->next && b->next->free) {
      Block* n = b->next;
      erase_free(n);
      b->size += n->size;
      b->next = n->next;
      if (n->next) n->next->prev = b;
      delete n;
    }
    if (b->prev && b->prev->free) {
      Block* p0 = b->prev;
      erase_free(p0);
      p0->size += b->size;
      p0->next = b->next;
      if (b->next) b->next->prev = p0;
      delete b;
      b = p0;
    }
    free_.emplace(b->size, b);
  }

  // Return fully idle chunks to the system; returns bytes released.
  size_t release_idle() {
    std::lock_guard<std::mutex> g(mu_);
    size_t freed = 0;
    std::vector<Chunk*> keep;
    for (Chunk* c : chunks_) {
      Block* h = c->head;
      if (h->free && h->next == nullptr && h->size == c->size) {
        erase_free(h);
        delete h;
        freed += c->size;
        reserved_ -= c->size;
        free_chunk(c);
      } else {
        keep.push_back(c);
      }
    }
    chunks_.swap(keep);
    return freed;
  }

  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    d["allocated"] = allocated_;
    d["reserved"] = reserved_;
    d["peak_allocated"] = peak_;
    d["chunks"] = chunks_.size();
    d["free_blocks"] = free_.size();
    d["live_blocks"] = live_.size();
    d["num_allocs"] = n_alloc_;
    d["reuse_hits"] = hits_;
    d["pinned"] = pinned();
    return d;
  }

 private:
  struct Chunk;
  struct Block {
    char* ptr;
    size_t size;
    bool free;
    Block* prev;
    Block* next;
    Chunk* chunk;
  };
  struct Chunk {
    char* base;
    size_t size;
    bool pinned;
    Block* head;
  };

  size_t round_up(size_t n) const { return (n + align_ - 1) / align_ * align_; }

  Block* grow(size_t need) {
    const size_t sz = need > chunk_bytes_ ? round_up(need) : chunk_bytes_;
    void* p = nullptr;
    bool pinned_mem = false;
    if (hip_.alloc && hip_.alloc(&p, sz, 0) == 0 && p) {
      pinned_mem = true;
    } else {
      p = nullptr;
      if (posix_memalign(&p, 4096, sz) != 0) return nullptr;
    }
    Chunk* c = new Chunk{static_cast<char*>(p), sz, pinned_mem, nullptr};
    Block* b = new Block{c->base, sz, true, nullptr, nullptr, c};
    c->head = b;
    chunks_.push_back(c);
    reserved_ += sz;
    return b;
  }

  void split(Block* b, size_t need) {
    if (b->size - need < align_) return;
    Block* r = new Block{b->ptr + need, b->size - need, true, b, b->next, b->chunk};
    if (b->next) b->next->prev = r;
    b->next = r;
    b->size = need;
    free_.emplace(r->size, r);
  }

  void erase_free(Block* b) {
    auto range = free_.equal_range(b->size);
    for (auto it = range.first; it != range.second; ++it) {
      if (it->second == b) {
        free_.erase(it);
        return;
      }
    }
  }

  void free_chunk(Chunk* c) {
    if (c->pinned && hip_.release) hip_.release(c->base);
    else if (!c->pinned) std::free(c->base);
    delete c;
  }

  std::mutex mu_;
  size_t chunk_bytes_, align_;
  HipHost hip_;
  std::multimap<size_t, Block*> free_;
  std::unordered_map<char*, Block*> live_;
  std::vector<Chunk*> chunks_;
  size_t allocated_ = 0, reserved_ = 0, peak_ = 0, n_alloc_ = 0, hits_ = 0;
};

}  // namespace

void register_pinned_pool(py::module& m) {
  py::class_<PinnedPool>(m, "PinnedPool")
      .def(py::init<size_t, size_t, bool>(), py::arg("chunk_bytes") = 64u << 20, py::arg("alignment") = 256,
           py::arg("use_hip") = true)
      .def("allocate", &PinnedPool::allocate, py::arg("nbytes"), py::call_guard<py::gil_scoped_release>())
      .def("deallocate", &PinnedPool::deallocate, py::arg("ptr"), py::call_guard<py::gil_scoped_release>())
      .def("release_idle", &PinnedPool::release_idle)
      .def("stats", &PinnedPool::stats)
      .def_property_readonly("pinned", &PinnedPool::pinned);
}
