"""Generate paddlepaddle_amd/_compat_paths.py: the reference's internal module paths (``paddle.a.b.c``) whose every
public name (the module's ``__all__``, else its top-level public defs / classes) this package already implements in
the nearest importable ancestor package. Those paths import here as alias modules, so code written against the
reference's file layout (``from paddle.incubate.nn.functional.fused_rms_norm import fused_rms_norm``,
``from paddle.distributed.communication.group import Group``) runs unchanged.

Reads the reference tree's syntax only (ast, names) — no code is taken from it. Usage:
    python tools/gen_compat_paths.py [/root/reference/python/paddle]
"""
import ast
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SKIP = ("fluid", "base", "cinn", "tensorrt", "pir", "libs", "proto", "tests", "test", "include", "_typing",
        "utils/gast", "jit/sot", "framework/ir", "incubate/xpu", "distributed/ps", "distributed/fleet/runtime",
        "distributed/passes/ps", "incubate/distributed/fleet")


# user-facing modules covered partially below the half mark: the alias still carries their implemented names
USER_FACING = {"amp.auto_cast", "distributed.fleet.recompute.recompute", "distributed.fleet.meta_parallel.pipeline_parallel",
               "distributed.fleet.meta_parallel.sharding.group_sharded_stage3",
               "distributed.fleet.meta_parallel.sharding.group_sharded_stage2",
               "distributed.fleet.meta_parallel.sharding.group_sharded_optimizer_stage2",
               "distributed.fleet.meta_parallel.pp_utils.utils", "distributed.fleet.utils.log_util",
               "distributed.fleet.meta_parallel.parallel_layers.random", "nn.functional.flash_attention"}


# names found in ANOTHER module of this package are bound only where checked by hand to be the same API (a bare
# name match is not enough: shufflenetv2.InvertedResidual is not mobilenet's, utils.flops.flops is not hapi's)
SAME_API = {
    "distributed.fleet.meta_parallel.parallel_layers": {"RNGStatesTracker"},
    "distributed.fleet.meta_parallel.parallel_layers.random": {"RNGStatesTracker"},
    "distributed.io": {"is_persistable", "load_persistables", "save_persistables"},
    "framework.framework": {"get_default_dtype", "set_default_dtype"},
    "hapi.hub": {"help", "list"},
    "incubate.autograd.primitives": None,  # every name: the paddle tensor op of that name
    "incubate.nn.loss": {"identity_loss"},
    "incubate.nn.memory_efficient_attention": {"memory_efficient_attention"},
    "jit.api": {"HookRemoveHelper"},
    "nn.initializer.lazy_init": {"LazyGuard"},
    "nn.quant.qat": {"QuantedConv2D", "QuantedLinear"},
    "nn.quant.qat.conv": {"QuantedConv2D"},
    "nn.quant.qat.linear": {"QuantedLinear"},
    "optimizer.lbfgs": {"dot"},
    "quantization.observers.abs_max": {"AbsmaxObserverLayer"},
    "quantization.observers.groupwise": {"GroupWiseWeightObserverLayer"},
    "quantization.quanters.abs_max": {"FakeQuanterWithAbsMaxObserverLayer"},
    "static.amp.debugging": {"collect_operator_stats"},
    "static.nn.common": {"ExponentialMovingAverage"},
    "static.nn.metric": {"auc", "ctr_metric_bundle"},
    "static.nn.sequence_lod": {"sequence_mask"},
    "tensor.attribute": None,
}


def public_names(path):
    tree = ast.parse(open(path).read())
    alln, defs, reexp = None, [], []
    for node in tree.body:
        if isinstance(node, ast.ImportFrom) and (node.level > 0 or (node.module or "").startswith("paddle")):
            reexp += [a.asname or a.name for a in node.names if a.name != "*" and not (a.asname or a.name).startswith("_")]
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            try:
                alln = [str(n) for n in ast.literal_eval(node.value)]
            except Exception:  # noqa: BLE001 - computed __all__
                alln = None
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)) and not node.name.startswith("_"):
            defs.append(node.name)
    # an empty __all__ (names exported by the package): the public defs; a pure re-export module: what it imports
    return alln if alln else (defs or reexp)


def importable(name):
    try:
        return importlib.import_module(name)
    except Exception:  # noqa: BLE001
        return None


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/python/paddle"
    os.environ["PADDLE_AMD_NO_COMPAT_PATHS"] = "1"  # real modules only
    import paddlepaddle_amd  # noqa: F401
    table, extra = {}, {}
    index = {}  # public name -> {module defining the object}
    for mname, m in list(sys.modules.items()):
        if not mname.startswith("paddlepaddle_amd") or m is None:
            continue
        for n, o in list(vars(m).items()):
            if n.startswith("_") or isinstance(o, type(sys)):
                continue
            om = getattr(o, "__module__", None)
            if isinstance(om, str) and om.startswith("paddlepaddle_amd") and om == mname:
                index.setdefault(n, set()).add(mname)

    def elsewhere(n):
        c = index.get(n, set())
        return next(iter(c))[len("paddlepaddle_amd."):] if len(c) == 1 else None
    for root, _dirs, files in sorted(os.walk(ref)):
        rel = os.path.relpath(root, ref)
        if any(rel == s or rel.startswith(s + "/") for s in SKIP):
            continue
        for f in sorted(files):
            if not f.endswith(".py") or (f.startswith("_") and f != "__init__.py"):
                continue
            mod = f[:-3] if rel == "." else rel.replace("/", ".") + "." + f[:-3]
            if mod.endswith(".__init__"):
                mod = mod[:-len(".__init__")]
            parts = mod.split(".")
            if any(p.startswith("_") for p in parts) or importable("paddlepaddle_amd." + mod) is not None:
                continue
            try:
                names = public_names(os.path.join(root, f))
            except SyntaxError:
                continue
            if not names:
                continue
            for i in range(len(parts) - 1, 0, -1):  # nearest importable ancestor
                src = "paddlepaddle_amd." + ".".join(parts[:i])
                anc = importable(src)
                if anc is not None:
                    break
            else:
                continue
            have = sorted({n for n in names if hasattr(anc, n)})
            for n in sorted(set(names) - set(have)):  # implemented in another module of this package
                o = elsewhere(n)
                ok = mod in SAME_API and (SAME_API[mod] is None or n in SAME_API[mod])
                if o is not None and ok:
                    extra.setdefault(mod, {})[n] = o
            have = sorted(set(have) | set(extra.get(mod, {})))
            # every public name implemented, or (partial) at least half of them: the alias exposes what exists and
            # the table lists the rest
            if len(have) == len(set(names)) or (have and (2 * len(have) >= len(set(names)) or mod in USER_FACING)):
                table[mod] = (src[len("paddlepaddle_amd."):], have, sorted(set(names) - set(have)))
    out = os.path.join(ROOT, "paddlepaddle_amd", "_compat_paths.py")
    with open(out, "w") as fh:
        fh.write('"""Generated by tools/gen_compat_paths.py: reference module path -> (implementing package of this\n'
                 'framework, the reference module\'s public names implemented there). Installed as alias modules by\n'
                 'paddlepaddle_amd._compat_import. MISSING: public names of a partially covered module that\n'
                 'this framework does not implement under that path."""\n\nPATHS = {\n')
        for k in sorted(table):
            src, names, _miss = table[k]
            fh.write(f"    {k!r}: ({src!r}, {names!r}),\n")
        fh.write("}\n\n# names of an alias path implemented in another module of this framework\nEXTRA = {\n")
        for k in sorted(extra):
            if k in table:
                fh.write(f"    {k!r}: {extra[k]!r},\n")
        fh.write("}\n\nMISSING = {\n")
        for k in sorted(table):
            if table[k][2]:
                fh.write(f"    {k!r}: {table[k][2]!r},\n")
        fh.write("}\n")
    print(f"{len(table)} module paths -> {out}")


if __name__ == "__main__":
    main()
