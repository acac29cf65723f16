"""Run the reference's own docstring examples against paddlepaddle_amd and compare printed values.

The reference documents every public API with ``>>>`` examples and their expected output (printed by
PaddlePaddle itself). Those examples are the parity fixtures this repo has: each example block runs with
``import paddle`` resolved to ``paddlepaddle_amd``, and its output is compared with the documented one by a
tolerant checker (Tensor reprs compared by shape / dtype / stop_gradient / values at rtol 1e-5, atol 1e-6;
``place`` ignored, since the docs were printed on CPU or GPU at random; other text compared after whitespace
normalisation with the numbers compared numerically).

Examples that are not deterministic are not counted: any block that draws random numbers (``rand``,
``randn``, ``uniform``, ``normal``, ``dropout``, ...), needs a device or a cluster (xdoctest ``REQUIRES``),
or is marked ``+SKIP``. The outcome per example is one of pass / fail / error / skip; a failure after a
skipped example of the same docstring that raised NameError counts as "skip" (it depends on the skipped one).

Usage: python tools/ref_doctests.py [--ref /root/reference] [--modules tensor nn/functional ...] [-v]
Prints one summary line per module and the overall deterministic pass rate; ``--json`` writes the results.
"""
from __future__ import annotations

import argparse
import ast
import contextlib
import doctest
import importlib
import importlib.abc
import importlib.util
import io
import json
import math
import os
import re
import signal
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DEFAULT_MODULES = ["tensor", "nn/functional", "nn/layer", "fft.py", "signal.py", "linalg.py"]

_RANDOM = re.compile(
    r"\b(rand|randn|randint|randint_like|randperm|uniform|uniform_|normal|normal_|standard_normal|gaussian|"
    r"bernoulli|bernoulli_|multinomial|poisson|binomial|exponential_|cauchy_|geometric_|log_normal|"
    r"dropout|dropout2d|dropout3d|alpha_dropout|feature_alpha_dropout|rrelu|shuffle|random_split|"
    r"Dropout|Dropout2D|Dropout3D|AlphaDropout|RReLU|gumbel_softmax|sample|rsample|random|seed|"
    r"empty|empty_like|Uniform|Normal|XavierUniform|XavierNormal|KaimingUniform|KaimingNormal|"
    r"TruncatedNormal|Orthogonal)\s*\(")
_LAYER_INIT = re.compile(r"\bnn\.(Linear|Conv\dD|Conv\dDTranspose|Embedding|LSTM|GRU|SimpleRNN|RNN|BiRNN|"
                         r"MultiHeadAttention|Transformer\w*|Bilinear|BatchNorm\w*|LayerNorm|GroupNorm|"
                         r"InstanceNorm\w*|PReLU|SpectralNorm|LSTMCell|GRUCell|SimpleRNNCell|RMSNorm|"
                         r"LocalResponseNorm|SyncBatchNorm|Conv\dD\w*|Linear\w*)\s*\(")
_SHELL = re.compile(r"os\.system|subprocess|pip install|shutil\.rmtree|os\.remove|os\.unlink|urlopen|wget|"
                    r"download|get_path_from_url")
_REQUIRES = re.compile(r"REQUIRES\(env\s*:\s*(GPU|XPU|DISTRIBUTED|CUSTOM_DEVICE|IPU|TENSORRT|CINN)", re.I)


# ---------------------------------------------------------------------------------------------- import alias
class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """``import paddle[.x.y]`` -> ``paddlepaddle_amd[.x.y]`` (the same module objects)."""

    def find_spec(self, name, path=None, target=None):
        if name == "paddle" or name.startswith("paddle."):
            real = "paddlepaddle_amd" + name[len("paddle"):]
            try:
                importlib.import_module(real)
            except Exception:
                return None
            return importlib.util.spec_from_loader(name, self)
        return None

    def create_module(self, spec):
        return sys.modules["paddlepaddle_amd" + spec.name[len("paddle"):]]

    def exec_module(self, module):
        pass


def install_alias():
    if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _AliasFinder())
    import paddlepaddle_amd  # noqa: F401


# ---------------------------------------------------------------------------------------------- comparison
_F = r"(?:\d+\.?\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|nan|inf)"
_NUM = (r"(?:[-+]?" + _F + r"\s*[-+]\s*(?:" + _F + r")?j"      # complex a+bj (numpy prints 1.+1.j, python (1+1j))
        r"|[-+]?(?:" + _F + r")?j"                               # pure imaginary
        r"|[-+]?" + _F + r")")
_TOKEN = re.compile(r"True|False|" + _NUM)


def _numbers(s):
    out = []
    for tok in _TOKEN.findall(s):
        if tok in ("True", "False"):
            out.append(tok == "True")
            continue
        try:
            out.append(complex(tok.replace(" ", "")) if tok.endswith("j") else float(tok))
        except ValueError:
            pass
    return out


def _close(a, b, rtol=1e-5, atol=1e-6):
    if isinstance(a, bool) or isinstance(b, bool):
        return a == b
    if isinstance(a, complex) or isinstance(b, complex):
        return abs(complex(a) - complex(b)) <= atol + rtol * abs(complex(b))
    if math.isnan(a) and math.isnan(b):
        return True
    if math.isinf(a) or math.isinf(b):
        return a == b
    return abs(a - b) <= atol + rtol * abs(b)


def _split_tensors(s):
    """[(shape, dtype, stop_gradient, values)] for every Tensor repr in s, plus the text outside them."""
    tensors, rest, pos = [], [], 0
    for m in re.finditer(r"Tensor\(shape=\[([^\]]*)\],\s*dtype=([\w.]+),\s*place=(?:Place\([^)]*\)|\w*Place(?:\([^)]*\))?),\s*"
                         r"stop_gradient=(True|False),", s):
        rest.append(s[pos:m.start()])
        # the payload runs to the matching close paren of "Tensor("
        depth, i = 1, m.start() + len("Tensor(")
        while i < len(s) and depth:
            if s[i] in "([":
                depth += 1
            elif s[i] in ")]":
                depth -= 1
            i += 1
        payload = s[m.end():i - 1]
        dt = m.group(2).replace("paddle.", "")
        tensors.append((m.group(1).replace(" ", ""), dt, m.group(3), _numbers(payload)))
        pos = i
    rest.append(s[pos:])
    return tensors, "".join(rest)


def outputs_match(want, got):
    if want == got:
        return True
    w_t, w_rest = _split_tensors(want)
    g_t, g_rest = _split_tensors(got)
    if len(w_t) != len(g_t):
        return False
    for (ws, wd, wsg, wv), (gs, gd, gsg, gv) in zip(w_t, g_t):
        if ws != gs or wd != gd or wsg != gsg or len(wv) != len(gv):
            return False
        if not all(_close(g, w) for g, w in zip(gv, wv)):
            return False
    wn, gn = _numbers(w_rest), _numbers(g_rest)
    if len(wn) != len(gn) or not all(_close(g, w) for g, w in zip(gn, wn)):
        return False
    strip = lambda t: re.sub(r"[\s()]+", "", _TOKEN.sub("#", t))  # noqa: E731
    return strip(w_rest) == strip(g_rest)


# ---------------------------------------------------------------------------------------------- extraction
def _docstrings(path):
    """(qualified name, docstring) of every function / class / method with a ``>>>`` example."""
    with open(path, encoding="utf-8") as f:
        tree = ast.parse(f.read())
    out = []

    def visit(node, prefix):
        for ch in ast.iter_child_nodes(node):
            if isinstance(ch, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                name = f"{prefix}{ch.name}"
                doc = ast.get_docstring(ch, clean=True)
                if doc and ">>>" in doc:
                    out.append((name, doc))
                if isinstance(ch, ast.ClassDef):
                    visit(ch, name + ".")
    visit(tree, "")
    return out


class _Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise _Timeout()


_DIRECTIVE_LINE = re.compile(r"^(\s*)>>>\s*#\s*doctest:\s*(.*?)\s*$", re.M)


def _sentinelize(doc):
    """xdoctest directive lines (``>>> # doctest: +SKIP("why")``) -> a sentinel call the runner interprets;
    the plain doctest parser rejects them (directive on a line with no example / unknown option)."""
    return _DIRECTIVE_LINE.sub(lambda m: f"{m.group(1)}>>> __doctest_directive__({m.group(2)!r})", doc)


def _merge_continuations(examples):
    """xdoctest lets a statement continue on ``>>>`` lines (``>>> x = f([1,`` / ``>>>      2])``) and an
    ``else:`` / ``except:`` start a new ``>>>`` block: join an example that does not compile on its own with its
    neighbours (a dangling else joins the previous block, anything else the following ones) until it does."""
    def compiles(src):
        try:
            compile(src, "<merge>", "exec")
            return True
        except SyntaxError:
            return False

    out, i = [], 0
    while i < len(examples):
        ex = examples[i]
        src, first, j = ex.source, ex, i
        if out and re.match(r"(else|elif|except|finally)\b", src.lstrip()):
            first = out.pop()
            src = first.source + src
        while not compiles(src) and j + 1 < len(examples):
            j += 1
            src = src + examples[j].source
        last = examples[j]
        if src != ex.source:
            ex = doctest.Example(src, last.want, last.exc_msg, lineno=first.lineno, indent=first.indent,
                                 options=first.options)
        out.append(ex)
        i = j + 1
    return out


def _drop_text_blocks(doc):
    """Remove ``.. code-block:: text`` bodies: prompts inside them are pseudo-code, not examples."""
    out, skip_indent = [], None
    for line in doc.splitlines():
        stripped = line.lstrip()
        ind = len(line) - len(stripped)
        if skip_indent is not None:
            if not stripped or ind > skip_indent:
                continue
            skip_indent = None
        if re.match(r"\.\.\s+code-block::\s*(text|none|bash|shell|console)\s*$", stripped):
            skip_indent = ind
            continue
        out.append(line)
    return "\n".join(out)


def module_namespace(rel):
    """Names of our module matching a reference file, like xdoctest's default of running a docstring's
    examples in its module's globals (``jit/utils.py`` -> ``paddle.jit.utils``)."""
    mod = "paddle." + rel[:-3].replace("/", ".") if rel.endswith(".py") else None
    if mod is None:
        return {}
    try:
        m = importlib.import_module(mod)
    except Exception:
        return {}
    return {k: v for k, v in vars(m).items() if not k.startswith("_")}


def run_docstring(doc, name, timeout=20, base_globs=None):
    """[(status, source, want, got)] for each checked example of one docstring, executed in one namespace.

    xdoctest semantics: the output of statements without an expected output accumulates and is checked at
    the next statement that has one; ``+SKIP`` on its own line skips every statement up to ``-SKIP``."""
    if _REQUIRES.search(doc):
        return [("skip", "", "", "requires device")]
    parser = doctest.DocTestParser()
    doc = _drop_text_blocks(doc)
    try:
        examples = parser.get_examples(_sentinelize(doc), name)
    except ValueError as e:
        return [("error", "<parse>", "", f"unparsable docstring: {e}")]
    examples = _merge_continuations(examples)
    globs = dict(base_globs or {})
    globs.update({"__name__": "__doctest__", "__doctest_directive__": lambda *a: None})
    results, skipping, skipped_any, random_seen = [], False, False, False
    pending = ""
    for ex in examples:
        src = ex.source
        m = re.match(r"__doctest_directive__\((.*)\)\s*$", src.strip())
        if m:
            d = m.group(1)
            if "+SKIP" in d:
                skipping, pending = True, ""
            elif "-SKIP" in d:
                skipping, pending = False, ""
            if ex.want.strip():
                results.append(("skip", src, ex.want, "directive"))
            continue
        if skipping or re.search(r"doctest:\s*\+SKIP", src):
            skipped_any = True
            pending = ""
            if ex.want.strip():
                results.append(("skip", src, ex.want, "directive"))
            continue
        if _SHELL.search(src):  # examples that install packages or shell out are never executed
            results.append(("skip", src, ex.want, "shell"))
            skipped_any = True
            continue
        if _RANDOM.search(src) or (_LAYER_INIT.search(src) and "weight_attr" not in src):
            random_seen = True
        buf = io.StringIO()
        status, got = "pass", ""
        old = signal.signal(signal.SIGALRM, _alarm)
        signal.alarm(timeout)
        try:
            with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
                exec(compile(src, f"<{name}>", "single" if ex.want.strip() else "exec"), globs)
            got = buf.getvalue()
        except _Timeout:
            status, got = "error", "timeout"
        except BaseException as e:  # noqa: BLE001 - the example's own failure is the result
            got = buf.getvalue()
            if ex.exc_msg is not None:
                status = "pass"
            elif isinstance(e, NameError) and skipped_any:
                status = "skip"
            elif re.search(r"no network|needs network access", str(e)):
                # a dataset / hub download the offline image cannot make: environment-bound
                status, skipped_any = "skip", True
            elif isinstance(e, ModuleNotFoundError) and not str(e.name or "").startswith("paddle"):
                # a third-party package the image lacks (cv2, astor): environment-bound, like a device
                status, skipped_any = "skip", True
            else:
                status, got = "error", f"{type(e).__name__}: {e}"[:300]
        finally:
            signal.alarm(0)
            signal.signal(signal.SIGALRM, old)
        if status == "pass" and not ex.want.strip():
            pending += got
            continue
        if status == "pass" and ex.exc_msg is None:
            got = pending + got
            if not outputs_match(ex.want.strip(), got.strip()):
                status = "fail"
        pending = ""
        if status in ("fail", "error") and random_seen:
            status = "skip"  # depends on random numbers drawn earlier in this docstring
        results.append((status, src, ex.want, got))
    return results


def iter_files(ref, modules):
    base = os.path.join(ref, "python", "paddle")
    for m in modules:
        p = os.path.join(base, m)
        if os.path.isdir(p):
            for fn in sorted(os.listdir(p)):
                if fn.endswith(".py") and not fn.startswith("_"):
                    yield os.path.join(m, fn), os.path.join(p, fn)
        elif os.path.isfile(p):
            yield m, p


def run(ref="/root/reference", modules=None, verbose=False):
    install_alias()
    import numpy as np
    import paddlepaddle_amd as paddle
    np.set_printoptions(precision=8)
    per_module = {}
    failures = []
    for rel, path in iter_files(ref, modules or DEFAULT_MODULES):
        counts = {"pass": 0, "fail": 0, "error": 0, "skip": 0}
        base = module_namespace(rel)
        for name, doc in _docstrings(path):
            np.set_printoptions(precision=8, threshold=1000, edgeitems=3, linewidth=75, suppress=False)
            import torch
            torch.set_printoptions(profile="default")
            torch.set_grad_enabled(True)
            paddle.set_default_dtype("float32")
            if hasattr(paddle, "disable_static"):
                paddle.disable_static()
            # each reference example runs in a fresh process: reset the process-wide state examples set
            from paddlepaddle_amd.static import executor as _sx
            _sx._reset_default_programs()
            from paddlepaddle_amd.nn.layer import layers as _ly
            _ly._layer_name_counters.clear()
            _ly._param_name_counters.clear()
            if hasattr(paddle, "vision"):
                paddle.vision.set_image_backend("pil")
            for status, src, want, got in run_docstring(doc, f"{rel}:{name}", base_globs=base):
                counts[status] += 1
                if status in ("fail", "error"):
                    failures.append({"where": f"{rel}:{name}", "status": status, "source": src.strip()[:400],
                                     "want": want.strip()[:400], "got": got.strip()[:400]})
        per_module[rel] = counts
        if verbose:
            print(f"{rel:40s} {counts}", flush=True)
    tot = {k: sum(c[k] for c in per_module.values()) for k in ("pass", "fail", "error", "skip")}
    det = tot["pass"] + tot["fail"] + tot["error"]
    rate = tot["pass"] / det if det else 1.0
    return {"total": tot, "deterministic": det, "pass_rate": rate, "modules": per_module, "failures": failures}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--modules", nargs="*", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--show", type=int, default=0, help="print the first N failures")
    a = ap.parse_args()
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:  # examples that save files write them here
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            res = run(a.ref, a.modules, a.verbose)
        finally:
            os.chdir(cwd)
    t = res["total"]
    print(f"reference doc examples: {t['pass']} pass / {t['fail']} fail / {t['error']} error "
          f"({t['skip']} skipped as non-deterministic or device-bound); deterministic pass rate "
          f"{res['pass_rate'] * 100:.1f}%")
    for f in res["failures"][:a.show]:
        print(f"--- {f['status']} {f['where']}\n{f['source']}\n  want: {f['want']}\n  got:  {f['got']}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
