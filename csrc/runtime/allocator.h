// Auto-growth best-fit device allocator with stream-ordered reuse (header-only core).
//
// Reference behaviour: paddle/phi/core/memory/allocation/auto_growth_best_fit_allocator.cc (chunks grown
// on demand, best-fit block search, split + neighbour coalescing, free chunks released on OOM) and
// stream_safe_cuda_allocator.cc (a block freed on one stream is reused by another only after that
// stream's work on it has finished).
//
// Design for MI355X (288 GB HBM3E): a chunk is at least `min_chunk` (default 64 MiB) so the tens of
// thousands of activation / gradient buffers of a training step are carved from a few hundred hipMalloc
// regions, never returned to the driver in steady state. Every block belongs to the stream it was
// allocated on; a free puts it back in that stream's best-fit set at once (stream order makes the reuse
// safe). When a stream finds nothing to fit it may take a free block of another stream: an event recorded
// on the owner stream is waited on by the requester (device-side wait, no host sync) before the memory is
// handed out. Raw memory and events come through a Backend of function pointers, so the same code runs on
// HIP (allocator_hip.cpp) and on host memory for the CPU unit tests.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

namespace pa_alloc {

struct Backend {
  void* (*raw_alloc)(size_t bytes, int device);       // nullptr on failure
  void (*raw_free)(void* p, int device);
  void (*cross_stream_wait)(uintptr_t owner, uintptr_t user, int device);  // user waits for owner's work
  void (*sync_device)(int device);
};

struct Stats {
  int64_t allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  int64_t n_alloc = 0, n_free = 0, n_chunks = 0, n_raw_alloc = 0, n_raw_free = 0, n_cross_stream = 0;
  int64_t n_oom_release = 0;
};

class BestFitAllocator {
 public:
  static constexpr size_t kAlign = 512;
  static constexpr uintptr_t kPoolBit = uintptr_t(1) << 63;

  BestFitAllocator(Backend be, int device, size_t min_chunk = size_t(64) << 20)
      : be_(be), device_(device), min_chunk_(min_chunk) {}

  ~BestFitAllocator() { release_all(); }

  // Graph capture: while `stream` is being captured its allocations come from the private pool
  // `pool_id`, whose free blocks are never handed to other streams / pools, so the addresses a captured
  // graph uses stay reserved for its replays (reference: CUDA graph memory pools). end_pool stops the
  // redirection; release_pool returns the pool's blocks to ordinary use once the graph is gone.
  // A pool may be shared by several graphs: every begin_pool takes a reference that release_pool drops, and
  // the pool's memory returns to ordinary use only when the last graph using it is gone.
  void begin_pool(uintptr_t stream, uint64_t pool_id) {
    std::lock_guard<std::mutex> g(mu_);
    const uintptr_t pkey = kPoolBit | static_cast<uintptr_t>(pool_id);
    capture_[stream] = pkey;
    if (pool_origin_.find(pkey) == pool_origin_.end()) pool_origin_[pkey] = stream;
    ++pool_refs_[pkey];
    released_.erase(pkey);  // a reused pool id: frees during this capture stay in the pool
  }

  void end_pool(uintptr_t stream) {
    std::lock_guard<std::mutex> g(mu_);
    capture_.erase(stream);
  }

  void release_pool(uint64_t pool_id) {
    std::lock_guard<std::mutex> g(mu_);
    const uintptr_t pkey = kPoolBit | static_cast<uintptr_t>(pool_id);
    auto o = pool_origin_.find(pkey);
    if (o == pool_origin_.end()) return;
    auto rc = pool_refs_.find(pkey);
    if (rc != pool_refs_.end() && --rc->second > 0) return;  // another graph still replays into this pool
    pool_refs_.erase(pkey);
    const uintptr_t dst = o->second;
    released_[pkey] = dst;
    auto pit = pools_.find(pkey);
    if (pit != pools_.end()) {
      std::vector<Key> keys(pit->second.begin(), pit->second.end());
      pools_.erase(pit);
      for (const Key& k : keys) {
        Block* b = lookup(k);
        b->stream = dst;
        b = coalesce(b);
        pools_[dst].insert(key(b));
      }
    }
    pool_origin_.erase(o);
  }

  void* allocate(size_t bytes, uintptr_t stream_in) {
    std::lock_guard<std::mutex> g(mu_);
    const size_t need = round(bytes ? bytes : 1);
    auto cap = capture_.find(stream_in);
    const uintptr_t stream = cap == capture_.end() ? stream_in : cap->second;
    Block* b = take(need, stream);
    if (b == nullptr && cap == capture_.end()) b = take_other_stream(need, stream);
    if (b == nullptr) {
      Chunk* c = grow(need, stream);
      if (c == nullptr && cap != capture_.end()) return nullptr;  // no device sync inside a capture
      if (c == nullptr) {
        release_locked();
        ++st_.n_oom_release;
        c = grow(need, stream);
        if (c == nullptr) return nullptr;
      }
      b = c->head;
      pools_[stream].erase(key(b));
    }
    split(b, need, stream);
    b->free = false;
    live_[b->ptr] = b;
    st_.allocated += static_cast<int64_t>(b->size);
    st_.peak_allocated = std::max(st_.peak_allocated, st_.allocated);
    ++st_.n_alloc;
    return b->ptr;
  }

  // returns false for a pointer this allocator does not own
  bool deallocate(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(static_cast<char*>(p));
    if (it == live_.end()) return false;
    Block* b = it->second;
    live_.erase(it);
    st_.allocated -= static_cast<int64_t>(b->size);
    ++st_.n_free;
    b->free = true;
    auto rel = released_.find(b->stream);
    if (rel != released_.end()) b->stream = rel->second;  // its graph pool is gone: back to the stream
    b = coalesce(b);
    pools_[b->stream].insert(key(b));
    return true;
  }

  // give every completely free chunk back to the driver (reference: Release / FreeIdleChunks)
  size_t release_free_chunks() {
    std::lock_guard<std::mutex> g(mu_);
    return release_locked();
  }

  Stats stats() {
    std::lock_guard<std::mutex> g(mu_);
    return st_;
  }

  void reset_peaks() {
    std::lock_guard<std::mutex> g(mu_);
    st_.peak_allocated = st_.allocated;
    st_.peak_reserved = st_.reserved;
  }

  size_t block_size(void* p) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(static_cast<char*>(p));
    return it == live_.end() ? 0 : it->second->size;
  }

  // number of free blocks over all streams (fragmentation diagnostics / tests)
  size_t free_blocks() {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (auto& kv : pools_) n += kv.second.size();
    return n;
  }

 private:
  size_t release_locked() {
    be_.sync_device(device_);
    size_t freed = 0;
    for (auto it = chunks_.begin(); it != chunks_.end();) {
      Chunk* c = it->second;
      Block* h = c->head;
      // a free chunk of a live graph pool is not idle: the graph's replays still read and write it
      const bool live_pool = (h->stream & kPoolBit) && pool_origin_.count(h->stream);
      if (h->free && h->next == nullptr && h->size == c->size && !live_pool) {
        pools_[h->stream].erase(key(h));
        be_.raw_free(c->base, device_);
        freed += c->size;
        st_.reserved -= static_cast<int64_t>(c->size);
        --st_.n_chunks;
        ++st_.n_raw_free;
        blocks_.erase(h->ptr);
        delete h;
        delete c;
        it = chunks_.erase(it);
      } else {
        ++it;
      }
    }
    return freed;
  }

  struct Chunk;
  struct Block {
    char* ptr;
    size_t size;
    bool free;
    Block* prev;
    Block* next;
    Chunk* chunk;
    uintptr_t stream;
  };
  struct Chunk {
    char* base;
    size_t size;
    Block* head;
  };
  using Key = std::pair<size_t, char*>;  // best fit: smallest size, then lowest address

  static size_t round(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }
  static Key key(Block* b) { return {b->size, b->ptr}; }

  Block* lookup(const Key& k) { return blocks_.at(k.second); }

  Block* take(size_t need, uintptr_t stream) {
    auto pit = pools_.find(stream);
    if (pit == pools_.end()) return nullptr;
    auto& pool = pit->second;
    auto it = pool.lower_bound({need, nullptr});
    if (it == pool.end()) return nullptr;
    Block* b = lookup(*it);
    pool.erase(it);
    return b;
  }

  Block* take_other_stream(size_t need, uintptr_t stream) {
    Block* best = nullptr;
    uintptr_t owner = 0;
    for (auto& kv : pools_) {
      if (kv.first == stream || (kv.first & kPoolBit)) continue;  // graph pools are never shared
      auto it = kv.second.lower_bound({need, nullptr});
      if (it == kv.second.end()) continue;
      if (best == nullptr || it->first < best->size) {
        best = lookup(*it);
        owner = kv.first;
      }
    }
    if (best == nullptr) return nullptr;
    pools_[owner].erase(key(best));
    be_.cross_stream_wait(owner, stream, device_);  // the requester waits for the owner's pending work
    ++st_.n_cross_stream;
    best->stream = stream;
    return best;
  }

  Chunk* grow(size_t need, uintptr_t stream) {
    size_t sz = need < min_chunk_ ? min_chunk_ : need;
    sz = (sz + (size_t(2) << 20) - 1) / (size_t(2) << 20) * (size_t(2) << 20);  // 2 MiB granules
    void* p = be_.raw_alloc(sz, device_);
    if (p == nullptr && sz > need) {
      sz = round(need);
      p = be_.raw_alloc(sz, device_);
    }
    if (p == nullptr) return nullptr;
    ++st_.n_raw_alloc;
    Chunk* c = new Chunk{static_cast<char*>(p), sz, nullptr};
    Block* b = new Block{c->base, sz, true, nullptr, nullptr, c, stream};
    c->head = b;
    blocks_[b->ptr] = b;
    chunks_[c->base] = c;
    pools_[stream].insert(key(b));
    st_.reserved += static_cast<int64_t>(sz);
    st_.peak_reserved = std::max(st_.peak_reserved, st_.reserved);
    ++st_.n_chunks;
    return c;
  }

  void split(Block* b, size_t need, uintptr_t stream) {
    if (b->size - need < kAlign) return;
    Block* r = new Block{b->ptr + need, b->size - need, true, b, b->next, b->chunk, stream};
    blocks_[r->ptr] = r;
    if (b->next) b->next->prev = r;
    b->next = r;
    b->size = need;
    pools_[stream].insert(key(r));
  }

  Block* coalesce(Block* b) {
    // merge with free neighbours of the same stream (their pending work is ordered with ours)
    Block* n = b->next;
    if (n && n->free && n->stream == b->stream) {
      pools_[n->stream].erase(key(n));
      b->size += n->size;
      b->next = n->next;
      if (n->next) n->next->prev = b;
      blocks_.erase(n->ptr);
      delete n;
    }
    Block* p = b->prev;
    if (p && p->free && p->stream == b->stream) {
      pools_[p->stream].erase(key(p));
      p->size += b->size;
      p->next = b->next;
      if (b->next) b->next->prev = p;
      blocks_.erase(b->ptr);
      delete b;
      b = p;
    }
    return b;
  }

  void release_all() {
    for (auto& kv : chunks_) {
      Chunk* c = kv.second;
      for (Block* b = c->head; b != nullptr;) {
        Block* nx = b->next;
        delete b;
        b = nx;
      }
      be_.raw_free(c->base, device_);
      delete c;
    }
    chunks_.clear();
    pools_.clear();
    live_.clear();
    blocks_.clear();
  }

  Backend be_;
  int device_;
  size_t min_chunk_;
  std::mutex mu_;
  std::map<char*, Chunk*> chunks_;
  std::unordered_map<uintptr_t, std::set<Key>> pools_;
  std::unordered_map<char*, Block*> live_;    // allocated blocks
  std::unordered_map<char*, Block*> blocks_;  // every block (free or not) by address
  std::unordered_map<uintptr_t, uintptr_t> capture_;      // capturing stream -> graph pool key
  std::unordered_map<uintptr_t, uintptr_t> pool_origin_;  // graph pool key -> its capturing stream
  std::unordered_map<uintptr_t, uintptr_t> released_;     // released pool key -> stream its blocks rejoin
  std::unordered_map<uintptr_t, int> pool_refs_;          // graph pool key -> graphs captured into it
  Stats st_;
};

}  // namespace pa_alloc
