// Eager backward engine: the graph traversal, dependency counting, gradient buffering and hook dispatch of a
// backward pass, run natively over the grad nodes the op library records (per-op backward functions: the
// hand-written HIP kernels' autograd functions and ATen's derivative formulas).
//
// Mirrors the reference's RunBackward (paddle/fluid/eager/backward.cc:105): getInDegreeMap over the reachable
// grad-node graph, a ready queue fed when a node's in-degree drops to zero, a per-node gradient holder that sums
// every contribution to an input slot (GradTensorHolder) before the node runs, gradient hooks applied to the
// summed slot, and for paddle.grad (general_grad.h) pruning to the nodes that lie on a path to a requested input
// plus capture of that input's gradient instead of accumulation into .grad.
//
// Python side: paddlepaddle_amd/autograd/engine.py builds the roots / captures / hook table and picks this
// engine under FLAGS_eager_backward_engine=native.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <deque>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

struct GNode {
  py::object fn;                              // the grad node (C++ node or Python Function backward object)
  std::vector<std::pair<int64_t, int>> next;  // per output slot: (node index or -1, input slot of that node)
  std::vector<py::object> buf;                // summed incoming gradients, one per input slot
  int indeg = 0;
  bool needed = true;                         // on a path to a captured input (paddle.grad) / always for backward
  bool is_py = false;                         // Python Function backward: zero-fill undefined slots
  int nslots = 0;
};

class Graph {
 public:
  int64_t index_of(const py::object& fn) {
    auto key = fn.ptr();
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    int64_t id = static_cast<int64_t>(nodes_.size());
    ids_.emplace(key, id);
    GNode n;
    n.fn = fn;
    nodes_.push_back(std::move(n));
    return id;
  }
  int64_t find(PyObject* p) const {
    auto it = ids_.find(p);
    return it == ids_.end() ? -1 : it->second;
  }
  std::vector<GNode> nodes_;

 private:
  std::unordered_map<PyObject*, int64_t> ids_;
};

py::object add_grads(const py::object& a, const py::object& b) {
  if (a.is_none()) return b;
  if (b.is_none()) return a;
  PyObject* r = PyNumber_Add(a.ptr(), b.ptr());
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

// roots:    [(node, slot, grad)]   gradient seeds (loss tensors' gradient edges)
// captures: [(node, slot)]         paddle.grad inputs: their summed gradient is returned, their node not run
//                                  unless another capture needs it; empty = backward() (run every node)
// hooks:    {(node, slot): [fn]}   gradient hooks, applied in order to the summed slot gradient
// helpers:  (zeros_for(node, slot), fix(grad, next_node, next_slot), is_py(node))
py::list run_backward(py::list roots, py::list captures, py::dict hooks, py::tuple helpers) {
  py::object zeros_for = helpers[0], fix = helpers[1], is_py_fn = helpers[2];
  Graph g;
  // ---- discovery + in-degree map (backward.cc getInDegreeMap): one count per incoming edge
  std::deque<int64_t> todo;
  for (auto r : roots) {
    auto t = r.cast<py::tuple>();
    g.index_of(t[0]);
  }
  for (size_t i = 0; i < g.nodes_.size(); ++i) todo.push_back(static_cast<int64_t>(i));
  while (!todo.empty()) {
    int64_t id = todo.front();
    todo.pop_front();
    py::object nf = g.nodes_[id].fn.attr("next_functions");
    std::vector<std::pair<int64_t, int>> next;
    for (auto e : nf) {
      auto et = e.cast<py::tuple>();
      if (et[0].is_none()) {
        next.emplace_back(-1, 0);
        continue;
      }
      int64_t before = static_cast<int64_t>(g.nodes_.size());
      int64_t j = g.index_of(py::reinterpret_borrow<py::object>(et[0]));
      if (j >= before) todo.push_back(j);
      next.emplace_back(j, et[1].cast<int>());
    }
    g.nodes_[id].next = std::move(next);
  }
  const int64_t n = static_cast<int64_t>(g.nodes_.size());
  for (int64_t i = 0; i < n; ++i)
    for (auto& e : g.nodes_[i].next)
      if (e.first >= 0) g.nodes_[e.first].indeg++;
  for (int64_t i = 0; i < n; ++i) {
    auto& nd = g.nodes_[i];
    nd.nslots = static_cast<int>(py::len(nd.fn.attr("_input_metadata")));
    nd.buf.assign(std::max(nd.nslots, 1), py::none());
    nd.is_py = is_py_fn(nd.fn).cast<bool>();
  }

  // ---- paddle.grad pruning (general_grad.h): a node runs only if one of its successors is a captured node or
  // runs itself; captured nodes hand back their slot gradient
  std::vector<std::pair<int64_t, int>> cap;
  std::vector<char> is_cap(n, 0);
  for (auto c : captures) {
    auto t = c.cast<py::tuple>();
    int64_t id = g.find(t[0].ptr());
    cap.emplace_back(id, t[1].cast<int>());
    if (id >= 0) is_cap[id] = 1;
  }
  if (!cap.empty()) {
    // reverse topological pass: successors before predecessors (Kahn order over a copy of the in-degrees)
    std::vector<int> indeg(n);
    for (int64_t i = 0; i < n; ++i) indeg[i] = g.nodes_[i].indeg;
    std::vector<int64_t> order;
    std::deque<int64_t> q;
    for (int64_t i = 0; i < n; ++i)
      if (indeg[i] == 0) q.push_back(i);
    while (!q.empty()) {
      int64_t i = q.front();
      q.pop_front();
      order.push_back(i);
      for (auto& e : g.nodes_[i].next)
        if (e.first >= 0 && --indeg[e.first] == 0) q.push_back(e.first);
    }
    std::vector<char> reach(n, 0);  // node is, or leads to, a captured node
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
      auto& nd = g.nodes_[*it];
      bool r = is_cap[*it];
      bool run = false;
      for (auto& e : nd.next)
        if (e.first >= 0 && reach[e.first]) run = true;
      reach[*it] = r || run;
      nd.needed = run;
    }
  }

  // ---- seed the roots' gradient holders
  for (auto r : roots) {
    auto t = r.cast<py::tuple>();
    auto& nd = g.nodes_[g.find(t[0].ptr())];
    int slot = t[1].cast<int>();
    if (slot >= static_cast<int>(nd.buf.size())) nd.buf.resize(slot + 1, py::none());
    nd.buf[slot] = add_grads(nd.buf[slot], py::reinterpret_borrow<py::object>(t[2]));
  }

  std::vector<py::object> captured(cap.size(), py::none());
  std::deque<int64_t> ready;
  for (int64_t i = 0; i < n; ++i)
    if (g.nodes_[i].indeg == 0) ready.push_back(i);
  while (!ready.empty()) {
    int64_t id = ready.front();
    ready.pop_front();
    auto& nd = g.nodes_[id];
    // gradient hooks on the summed slots (GradNodeBase::ApplyGradientHooks)
    if (hooks.size()) {
      for (size_t s = 0; s < nd.buf.size(); ++s) {
        if (nd.buf[s].is_none()) continue;
        py::tuple key = py::make_tuple(nd.fn, static_cast<int>(s));
        if (!hooks.contains(key)) continue;
        for (auto h : hooks[key].cast<py::list>()) {
          py::object r = h(nd.buf[s]);
          if (!r.is_none()) nd.buf[s] = r;
        }
      }
    }
    if (is_cap[id])
      for (size_t k = 0; k < cap.size(); ++k)
        if (cap[k].first == id && cap[k].second < static_cast<int>(nd.buf.size())) captured[k] = nd.buf[cap[k].second];
    py::tuple outs;
    bool ran = false;
    if (nd.needed) {
      bool any = false;
      for (auto& b : nd.buf) any = any || !b.is_none();
      if (any) {
        py::tuple args(nd.nslots);
        for (int s = 0; s < nd.nslots; ++s) {
          py::object b = s < static_cast<int>(nd.buf.size()) ? nd.buf[s] : py::none();
          if (b.is_none() && nd.is_py) b = zeros_for(nd.fn, s);
          args[s] = b;
        }
        py::object r = nd.is_py ? nd.fn.attr("apply")(*args) : nd.fn(*args);
        outs = py::isinstance<py::tuple>(r) ? r.cast<py::tuple>() : py::make_tuple(r);
        ran = true;
      }
    }
    for (auto& b : nd.buf) b = py::none();  // release the holder as soon as the node has consumed it
    for (size_t k = 0; k < nd.next.size(); ++k) {
      auto e = nd.next[k];
      if (e.first < 0) continue;
      auto& nx = g.nodes_[e.first];
      if (ran && k < py::len(outs) && !outs[k].is_none()) {
        py::object gk = fix(outs[k], nx.fn, e.second);
        if (e.second >= static_cast<int>(nx.buf.size())) nx.buf.resize(e.second + 1, py::none());
        nx.buf[e.second] = add_grads(nx.buf[e.second], gk);
      }
      if (--nx.indeg == 0) ready.push_back(e.first);
    }
  }
  py::list res;
  for (auto& c : captured) res.append(c);
  return res;
}

}  // namespace

void register_autograd_engine(py::module& m) {
  m.def("run_backward", &run_backward, py::arg("roots"), py::arg("captures"), py::arg("hooks"), py::arg("helpers"),
        "Eager backward over the grad-node graph (RunBackward: in-degree map, ready queue, slot sums, hooks, "
        "paddle.grad pruning and capture)");
}
