// Native eager backward executor over the grad-node graph, in C++ end to end (no Python per node).
//
// Reference behaviour: paddle/fluid/eager/backward.cc:105 RunBackward — in-degree map over the reachable grad
// nodes, a ready queue fed as in-degrees drop to zero, per-node gradient holders that sum every contribution to
// an input slot before the node runs, gradient hooks on the summed slot, paddle.grad pruning (general_grad.h) to
// the nodes on a path to a requested input and capture of that input's gradient.
//
// The nodes are the grad functions the op library records (the HIP kernels' autograd functions and ATen's
// derivative formulas). This executor walks them through the C++ Node interface: next_edges() for the graph,
// operator() to run a node (Python-defined functions re-enter Python only inside their own apply), the input
// metadata to validate each produced gradient (dtype cast, sum-reduction of broadcast dims), release_variables()
// right after a node ran when the graph is not retained (saved activations are freed as the backward proceeds),
// and the hooks in torch's order: tensor pre-hooks and retains-grad hooks (Tensor.register_hook / retain_grad
// through either framework's API, Module full-backward hooks), node pre-hooks, the node, node post-hooks. The
// framework's own (node, slot) table is only filled when hooks are registered for the pybind fallback.
// It runs on the calling thread; each node runs on the stream its forward ran on (Node::stream(), as torch's
// engine does), gradients crossing streams are ordered by an event (producer -> consumer), and the caller's
// current stream waits for every stream the backward used before it returns: no device-thread hand-off.
//
// Python side: paddlepaddle_amd/autograd/engine.py (FLAGS_eager_backward_engine=native) passes the root tensors
// and seeds, the paddle.grad inputs, and the framework's gradient-hook table keyed by (grad node, slot).
#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/grad_mode.h>
#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/autograd/variable.h>
#include <c10/core/Event.h>
#include <c10/core/StreamGuard.h>
#include <c10/core/impl/VirtualGuardImpl.h>

#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;
using torch::autograd::Edge;
using torch::autograd::Node;
using torch::autograd::variable_list;

namespace {

struct XNode {
  std::shared_ptr<Node> fn;
  std::vector<std::pair<int64_t, uint32_t>> next;  // per output: (node index or -1, input slot of that node)
  variable_list buf;                                // summed incoming gradients, one per input slot
  int indeg = 0;
  bool needed = true;
};

struct XGraph {
  std::vector<XNode> nodes;
  std::unordered_map<Node*, int64_t> ids;

  int64_t index_of(const std::shared_ptr<Node>& fn) {
    auto it = ids.find(fn.get());
    if (it != ids.end()) return it->second;
    int64_t id = static_cast<int64_t>(nodes.size());
    ids.emplace(fn.get(), id);
    XNode n;
    n.fn = fn;
    n.buf.resize(fn->num_inputs());
    nodes.push_back(std::move(n));
    return id;
  }
  int64_t find(Node* p) const {
    auto it = ids.find(p);
    return it == ids.end() ? -1 : it->second;
  }
};

// consumer stream waits for the producer stream (InputBuffer::add's cross-stream rule)
void order_streams(const std::optional<c10::Stream>& producer, const std::optional<c10::Stream>& consumer) {
  if (!producer || !consumer || *producer == *consumer) return;
  c10::Event ev{producer->device_type()};
  ev.record(*producer);
  consumer->wait(ev);
}

c10::Stream current_stream(const c10::Stream& like) {
  c10::impl::VirtualGuardImpl impl(like.device_type());
  return impl.getStream(like.device());
}

// torch's call_tensor_pre_hooks: Tensor.register_hook hooks, then retain_grad hooks, over the summed inputs
variable_list tensor_pre_hooks(Node& fn, variable_list inputs) {
  for (const auto& h : fn.tensor_pre_hooks()) inputs = (*h)(inputs);
  for (const auto& kv : fn.retains_grad_hooks()) inputs = (*kv.second)(inputs);
  return inputs;
}

at::Tensor unpack(py::handle h) {
  if (!THPVariable_Check(h.ptr())) throw std::invalid_argument("expected a torch.Tensor");
  return THPVariable_Unpack(h.ptr());
}

void accumulate(at::Tensor& slot, const at::Tensor& g) {
  if (!g.defined()) return;
  slot = slot.defined() ? slot + g : g;
}

// validate_outputs: a gradient flowing into a node's input slot takes that slot's dtype and shape
at::Tensor fix(at::Tensor g, const Node& nx, uint32_t slot) {
  if (!g.defined() || slot >= nx.num_inputs()) return g;
  const auto& m = nx.input_metadata(slot);
  if (m.was_default_constructed()) return g;
  if (!m.is_same_shape(g)) {
    if (!m.is_expandable_to_shape(g))
      throw std::runtime_error(m.incompatible_shape_error_message(slot, g).str());
    g = m.reduce_grad(g);
  }
  auto want = m.grad_dtype();
  at::ScalarType st = want.has_value() ? *want : c10::typeMetaToScalarType(m.dtype());
  if (g.scalar_type() != st && (at::isFloatingType(st) || at::isComplexType(st))) g = g.to(st);
  return g;
}

// roots:    [(tensor, seed gradient)]
// captures: [tensor]                     paddle.grad inputs (empty: backward(), every reachable node runs)
// hooks:    {(grad node object, slot): [fn]}   the framework's gradient hooks, applied to the summed slot
py::list run_backward(py::list roots, py::list captures, py::dict hooks, bool keep_graph, bool create_graph) {
  XGraph g;
  for (auto r : roots) {
    auto t = r.cast<py::tuple>();
    at::Tensor v = unpack(t[0]);
    Edge e = torch::autograd::impl::gradient_edge(v);
    if (!e.function) throw std::runtime_error("backward: the tensor has no grad node (stop_gradient=True)");
    int64_t id = g.index_of(e.function);
    at::Tensor seed = t[1].is_none() ? at::ones_like(v, at::MemoryFormat::Preserve) : unpack(t[1]);
    if (e.input_nr >= g.nodes[id].buf.size()) g.nodes[id].buf.resize(e.input_nr + 1);
    accumulate(g.nodes[id].buf[e.input_nr], seed);
  }
  // ---- discovery + in-degree map
  for (size_t i = 0; i < g.nodes.size(); ++i) {
    std::shared_ptr<Node> fn = g.nodes[i].fn;  // copy: nodes may reallocate below
    std::vector<std::pair<int64_t, uint32_t>> next;
    const auto& edges = fn->next_edges();
    next.reserve(edges.size());
    for (const auto& e : edges) {
      if (!e.function) {
        next.emplace_back(-1, 0);
        continue;
      }
      next.emplace_back(g.index_of(e.function), e.input_nr);
    }
    g.nodes[i].next = std::move(next);
  }
  const int64_t n = static_cast<int64_t>(g.nodes.size());
  for (int64_t i = 0; i < n; ++i)
    for (auto& e : g.nodes[i].next)
      if (e.first >= 0) g.nodes[e.first].indeg++;

  // ---- paddle.grad pruning + capture targets
  std::vector<std::pair<int64_t, uint32_t>> cap;
  std::vector<char> is_cap(n, 0);
  for (auto c : captures) {
    Edge e = torch::autograd::impl::gradient_edge(unpack(c));
    int64_t id = e.function ? g.find(e.function.get()) : -1;
    cap.emplace_back(id, e.input_nr);
    if (id >= 0) is_cap[id] = 1;
  }
  if (!cap.empty()) {
    std::vector<int> indeg(n);
    for (int64_t i = 0; i < n; ++i) indeg[i] = g.nodes[i].indeg;
    std::vector<int64_t> order;
    std::deque<int64_t> q;
    for (int64_t i = 0; i < n; ++i)
      if (indeg[i] == 0) q.push_back(i);
    while (!q.empty()) {
      int64_t i = q.front();
      q.pop_front();
      order.push_back(i);
      for (auto& e : g.nodes[i].next)
        if (e.first >= 0 && --indeg[e.first] == 0) q.push_back(e.first);
    }
    std::vector<char> reach(n, 0);
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
      auto& nd = g.nodes[*it];
      bool run = false;
      for (auto& e : nd.next)
        if (e.first >= 0 && reach[e.first]) run = true;
      reach[*it] = is_cap[*it] || run;
      nd.needed = run;
    }
  }

  // framework hooks, keyed by the grad node's Python object (the node keeps a pointer to its wrapper)
  std::unordered_map<PyObject*, std::vector<std::pair<uint32_t, py::list>>> node_hooks;
  for (auto item : hooks) {
    auto key = item.first.cast<py::tuple>();
    node_hooks[key[0].ptr()].emplace_back(key[1].cast<uint32_t>(), item.second.cast<py::list>());
  }

  at::AutoGradMode grad_mode(create_graph);
  // streams: the seeds were produced on the caller's current stream; every stream a node runs on is recorded
  // so the caller's stream can wait for all of them at the end
  std::vector<c10::Stream> used;
  auto note_stream = [&](const std::optional<c10::Stream>& s) {
    if (!s) return;
    for (const auto& u : used)
      if (u == *s) return;
    used.push_back(*s);
  };
  for (int64_t i = 0; i < n; ++i) {
    if (g.nodes[i].indeg != 0) continue;
    auto s = g.nodes[i].fn->stream();
    if (s) order_streams(current_stream(*s), s);
  }
  std::vector<at::Tensor> captured(cap.size());
  std::deque<int64_t> ready;
  for (int64_t i = 0; i < n; ++i)
    if (g.nodes[i].indeg == 0) ready.push_back(i);
  while (!ready.empty()) {
    int64_t id = ready.front();
    ready.pop_front();
    auto& nd = g.nodes[id];
    Node& fn = *nd.fn;
    const std::optional<c10::Stream> stream = fn.stream();
    note_stream(stream);
    c10::OptionalStreamGuard guard(stream);
    if (!fn.tensor_pre_hooks().empty() || !fn.retains_grad_hooks().empty()) nd.buf = tensor_pre_hooks(fn, std::move(nd.buf));
    auto hk = node_hooks.empty() || fn.pyobj() == nullptr ? node_hooks.end() : node_hooks.find(fn.pyobj());
    if (hk != node_hooks.end()) {
      for (auto& sh : hk->second) {
        if (sh.first >= nd.buf.size() || !nd.buf[sh.first].defined()) continue;
        for (auto h : sh.second) {
          py::object r = h(py::reinterpret_steal<py::object>(THPVariable_Wrap(nd.buf[sh.first])));
          if (!r.is_none()) nd.buf[sh.first] = unpack(r);
        }
      }
    }
    if (is_cap[id])
      for (size_t k = 0; k < cap.size(); ++k)
        if (cap[k].first == id && cap[k].second < nd.buf.size()) captured[k] = nd.buf[cap[k].second];
    variable_list outs;
    bool ran = false;
    if (nd.needed) {
      bool any = false;
      for (auto& b : nd.buf) any = any || b.defined();
      if (any) {
        variable_list inputs = std::move(nd.buf);
        for (const auto& h : fn.pre_hooks()) inputs = (*h)(inputs);
        if (!keep_graph) fn.will_release_variables();
        if (fn.post_hooks().empty()) {
          outs = fn(std::move(inputs));
        } else {  // post-hooks see (grad outputs, grad inputs), as in torch's call_post_hooks
          variable_list copy = inputs;
          outs = fn(std::move(copy));
          for (const auto& h : fn.post_hooks()) outs = (*h)(outs, inputs);
        }
        if (!keep_graph) fn.release_variables();
        ran = true;
      }
    }
    nd.buf.clear();
    nd.buf.shrink_to_fit();
    for (size_t k = 0; k < nd.next.size(); ++k) {
      auto e = nd.next[k];
      if (e.first < 0) continue;
      auto& nx = g.nodes[e.first];
      if (ran && k < outs.size() && outs[k].defined()) {
        if (e.second >= nx.buf.size()) nx.buf.resize(e.second + 1);
        order_streams(stream, nx.fn->stream());
        accumulate(nx.buf[e.second], fix(outs[k], *nx.fn, e.second));
      }
      if (--nx.indeg == 0) ready.push_back(e.first);
    }
  }
  for (const auto& s : used) order_streams(s, current_stream(s));  // the caller's stream sees every gradient
  py::list res;
  for (auto& c : captured) {
    if (c.defined()) res.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(c)));
    else res.append(py::none());
  }
  return res;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native eager backward executor (RunBackward over the grad-node graph, C++ end to end)";
  m.def("run_backward", &run_backward, py::arg("roots"), py::arg("captures"), py::arg("hooks"),
        py::arg("keep_graph"), py::arg("create_graph"));
}
