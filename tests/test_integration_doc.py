"""INTEGRATION.md's ctypes stubs against the binding's declarations.

The stubs are what a PipelineDP maintainer would copy, so every
`lib.<fn>.argtypes = [...]` / `.restype = ...` they set must equal
`pipelinedp_amd._native.signatures()` (which mirrors include/pipelinedp_amd.h,
checked by tests/test_abi.py), and every `lib.<fn>(...)` call must pass as many
arguments as the C function takes.  CPU only: nothing is loaded or called.
"""
import ast
import ctypes
import os
import re

from pipelinedp_amd import _native as N

DOC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")


def _python_blocks():
    with open(DOC) as f:
        text = f.read()
    return re.findall(r"```python\n(.*?)```", text, flags=re.S)


def _lib_attr(node):
    """'pdp_x' for the expression `lib.pdp_x`, else None."""
    if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "lib":
        return node.attr
    return None


def _namespace():
    ns = {"ctypes": ctypes, "P": ctypes.POINTER, "vp": ctypes.c_void_p, "u64": ctypes.c_uint64,
          "i64": ctypes.c_int64, "i32": ctypes.c_int32}
    for name in ("BoundConfig", "PartitionAccumulators", "NoiseParams", "HistogramBins", "SelectConfig",
                 "MetricOp", "BoundStats", "BoundPlanInfo"):
        ns[name] = getattr(N, name)
    return ns


def _collect():
    decls, calls = [], []
    for block in _python_blocks():
        tree = ast.parse(block)
        for node in ast.walk(tree):
            if isinstance(node, ast.Assign) and len(node.targets) == 1:
                t = node.targets[0]
                if isinstance(t, ast.Attribute) and t.attr in ("argtypes", "restype"):
                    fn = _lib_attr(t.value)
                    if fn is not None:
                        decls.append((fn, t.attr, node.value))
            if isinstance(node, ast.Call):
                fn = _lib_attr(node.func)
                if fn is not None:
                    calls.append((fn, len(node.args) + len(node.keywords)))
    return decls, calls


def test_doc_has_stubs():
    decls, calls = _collect()
    assert len(decls) >= 6 and len(calls) >= 6
    assert {"pdp_bound_contributions", "pdp_reduce_partitions", "pdp_add_noise",
            "pdp_dataset_histograms"} <= {fn for fn, _ in calls}


def test_doc_argtypes_match_binding():
    sig = N.signatures()
    ns = _namespace()
    decls, _ = _collect()
    for fn, what, expr in decls:
        assert fn in sig, f"INTEGRATION.md declares unknown symbol {fn}"
        value = eval(compile(ast.Expression(expr), DOC, "eval"), ns)  # noqa: S307 (our own doc)
        res, args = sig[fn]
        if what == "argtypes":
            assert list(value) == list(args), f"{fn}: INTEGRATION.md argtypes {value} != binding {args}"
        else:
            assert value is res, f"{fn}: INTEGRATION.md restype {value} != binding {res}"


def test_doc_calls_have_c_arity():
    sig = N.signatures()
    _, calls = _collect()
    for fn, n_args in calls:
        assert fn in sig, f"INTEGRATION.md calls unknown symbol {fn}"
        assert n_args == len(sig[fn][1]), f"{fn}: INTEGRATION.md passes {n_args} args, C takes {len(sig[fn][1])}"


def test_binding_matches_header_arity():
    """Every prototype in the header takes as many parameters as the binding declares."""
    hdr = os.path.join(os.path.dirname(DOC), "include", "pipelinedp_amd.h")
    with open(hdr) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    protos = dict()
    for m in re.finditer(r"\b(?:int|const char\s*\*)\s+(pdp_\w+)\s*\(([^)]*)\)\s*;", text):
        params = m.group(2).strip()
        protos[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    sig = N.signatures()
    assert set(sig) <= set(protos), sorted(set(sig) - set(protos))
    for fn, (_, args) in sig.items():
        assert protos[fn] == len(args), f"{fn}: header {protos[fn]} params, binding {len(args)}"
