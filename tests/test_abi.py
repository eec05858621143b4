"""The C-ABI boundary (include/pipelinedp_amd.h) on the CPU: the library loads,
exports every declared entry point, its ctypes mirror has the C struct layout
and constants, and the host-only entry points (plan, workspace sizing, argument
validation, error reporting) behave.  No device work is launched."""
import ctypes
import os
import re
import subprocess

import pytest

from pipelinedp_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pipelinedp_amd.h")

STRUCTS = {
    "pdp_bound_config": N.BoundConfig,
    "pdp_bound_plan_info": N.BoundPlanInfo,
    "pdp_partition_accumulators": N.PartitionAccumulators,
    "pdp_select_config": N.SelectConfig,
    "pdp_metric_op": N.MetricOp,
    "pdp_histogram_bins": N.HistogramBins,
    "pdp_bound_stats": N.BoundStats,
}


def _header_text():
    with open(HEADER) as f:
        src = f.read()
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def declared_functions():
    return sorted(set(re.findall(r"\b(pdp_[a-z0-9_]+)\s*\(", _header_text())))


def declared_constants():
    return {m.group(1): int(m.group(2), 0) for m in
            re.finditer(r"#define\s+PDP_([A-Z0-9_]+)\s+\(?(-?(?:0x[0-9A-Fa-f]+|\d+))\)?", _header_text())}


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    return N.lib()


def test_every_declared_function_is_exported(lib):
    fns = declared_functions()
    assert len(fns) >= 13
    assert set(fns) == set(N.EXPORTED_SYMBOLS)
    for name in fns:
        assert hasattr(lib, name), name


def test_constants_match_header():
    consts = declared_constants()
    skip = {"ABI_VERSION"}
    checked = 0
    for name, value in consts.items():
        if name.startswith("E_") or name == "OK" or name in skip:
            continue
        py = name[:-4] if name.endswith("_MAX") else name
        if hasattr(N, py):
            assert getattr(N, py) == value, name
            checked += 1
    assert checked >= 25
    assert consts["ABI_VERSION"] == N.ABI_VERSION


def test_struct_layouts_match_c(tmp_path):
    """sizeof / offsetof of every ABI struct, compiled by gcc from the header,
    equal the ctypes mirror's."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pipelinedp_amd.h"', "int main(void) {"]
    for cname, cls in STRUCTS.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for field, _ in cls._fields_:
            lines.append(f'  printf("{cname} {field} %zu\\n", offsetof({cname}, {field}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = {}
    for line in out.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, cls in STRUCTS.items():
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for field, _ in cls._fields_:
            assert got[(cname, field)] == getattr(cls, field).offset, (cname, field)


def _cfg(**kw):
    c = N.BoundConfig()
    c.n_rows, c.n_privacy_ids, c.n_partitions = 100_000_000, 1_000_000, 100_000
    c.l0, c.linf, c.value_kind, c.flags = 8, 2, N.VALUE_F64, N.ACC_NSUM
    c.min_value, c.max_value, c.middle = 0.0, 10.0, 5.0
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_abi_version_and_plan(lib):
    assert lib.pdp_abi_version() == N.ABI_VERSION
    info = N.BoundPlanInfo()
    assert lib.pdp_bound_plan(ctypes.byref(_cfg()), ctypes.byref(info)) == 0
    assert info.algorithm == N.ALGO_BUCKETED and info.merge == N.MERGE_RANGES
    assert info.pk_bits == 17 and info.n_ranges == 49
    assert info.n_buckets << info.bucket_bits >= 1_000_000
    assert info.lds_bytes <= 160 * 1024
    assert 64 - info.rand_shift >= 24
    # forced global path and forced atomic merge resolve as asked
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(algorithm=N.ALGO_GLOBAL_SKETCH)), ctypes.byref(info)) == 0
    assert info.algorithm == N.ALGO_GLOBAL_SKETCH and info.n_buckets == 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(merge=N.MERGE_ATOMIC)), ctypes.byref(info)) == 0
    assert info.merge == N.MERGE_ATOMIC
    # > 1024 ranges of 2,048 partitions: the two-level range merge, <= 256
    # coarse ranges in the bucket kernel (P = 1e7: 153 of 65,536 partitions)
    for merge in (N.MERGE_AUTO, N.MERGE_RANGES):
        assert lib.pdp_bound_plan(ctypes.byref(_cfg(n_partitions=10_000_000, merge=merge)), ctypes.byref(info)) == 0
        assert info.merge == N.MERGE_RANGES and info.n_ranges == 153


def test_sieve_plan(lib):
    """Threshold sieve (Plan.sieve): AUTO picks t = (l0 + 3 sqrt(l0) + 3) / (0.6 rows per id)
    up to 0.35 (C3: 0.154, C2: 0.325; C4 with 10 rows per id: off), a forced value is
    clamped to 1/2, < 0 is off, and small (one-level) plans never sieve."""
    info = N.BoundPlanInfo()
    c3 = dict(n_rows=1_000_000_000, n_privacy_ids=10_000_000, n_partitions=1_000_000, l0=2, linf=1)
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3)), ctypes.byref(info)) == 0
    assert abs(info.sieve / 65536 - (2 + 3 * 2 ** 0.5 + 3) / 60) < 1e-4
    assert lib.pdp_bound_plan(ctypes.byref(_cfg()), ctypes.byref(info)) == 0  # C2
    assert abs(info.sieve / 65536 - (8 + 3 * 8 ** 0.5 + 3) / 60) < 1e-4
    c4 = dict(n_rows=125_000_000, n_privacy_ids=12_500_000, n_partitions=10_000_000, l0=4, linf=2)
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c4)), ctypes.byref(info)) == 0
    assert info.sieve == 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c4, sieve=4096)), ctypes.byref(info)) == 0
    assert info.sieve == 4096 and info.key_format == N.KEYS_PACKED64  # 8-byte level-2 records (row in the key)
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve=-1)), ctypes.byref(info)) == 0
    assert info.sieve == 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve=1 << 20)), ctypes.byref(info)) == 0
    assert info.sieve == 1 << 15
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(n_rows=1_000_000, n_privacy_ids=5000, sieve=4096)),
                              ctypes.byref(info)) == 0
    assert info.sieve == 0  # one bucket level: no tile-local level 1
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(merge=N.MERGE_ATOMIC, sieve=4096)), ctypes.byref(info)) == 0
    assert info.sieve == 0  # the fix-up appends pair records: range merge only
    # the side band: auto for t <= 1/4 at t2 = 2t (C3 yes, C2 no), forced on / off
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3)), ctypes.byref(info)) == 0
    assert info.band == 2 * info.sieve
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve_band=-1)), ctypes.byref(info)) == 0
    assert info.band == 0 and info.sieve > 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg()), ctypes.byref(info)) == 0  # C2
    assert info.band == 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(sieve_band=1)), ctypes.byref(info)) == 0
    assert info.band == 1 << 15  # 2t capped at 1/2
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve=-1)), ctypes.byref(info)) == 0
    assert info.band == 0
    # the sieve's workspace holds the fix-up state and twice the pair records
    on, off = ctypes.c_uint64(0), ctypes.c_uint64(0)
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(**c3)), ctypes.byref(on)) == 0
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(**c3, sieve=-1)), ctypes.byref(off)) == 0
    assert on.value > off.value


def test_workspace_bytes(lib):
    small, big = ctypes.c_uint64(0), ctypes.c_uint64(0)
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(n_rows=1000)), ctypes.byref(small)) == 0
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg()), ctypes.byref(big)) == 0
    assert 0 < small.value < big.value
    # bucketed, compact records: two levels of (4 B record + 4 B row), the
    # bucket kernel's candidate list (4 B key + 4 B index) + pair records
    # (8 B key + 8 B nsum per kept slot)
    assert big.value >= 100_000_000 * 24 + 1_000_000 * 8 * 16
    # + the sieve's side band: one 8 B (id, row) slot per row, and pair
    # records for the main launch and the band's two fix-up launches
    assert big.value < 100_000_000 * 34 + 3 * 1_000_000 * 8 * 16 + (64 << 20)
    wide = ctypes.c_uint64(0)
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(key_format=N.KEYS_WIDE)), ctypes.byref(wide)) == 0
    assert wide.value >= 100_000_000 * 36 + 1_000_000 * 8 * 16
    cb = ctypes.c_uint64(0)
    assert lib.pdp_compact_workspace_bytes(1 << 20, ctypes.byref(cb)) == 0 and cb.value > 0


@pytest.mark.parametrize("field,value,code,msg", [
    ("l0", -1, -4, b"l0"), ("linf", -1, -4, b"linf"),
    ("max_contributions", -1, -4, b"max_contributions"),
    ("n_rows", 1 << 32, -1, b"n_rows"), ("n_partitions", 0, -1, b"n_partitions"),
    ("n_privacy_ids", 0, -1, b"n_privacy_ids"), ("value_kind", 7, -1, b"value_kind"),
    ("algorithm", 9, -1, b"algorithm"), ("merge", 5, -1, b"merge"), ("key_format", 6, -1, b"key_format"),
])
def test_invalid_configs_are_rejected(lib, field, value, code, msg):
    info = N.BoundPlanInfo()
    rc = lib.pdp_bound_plan(ctypes.byref(_cfg(**{field: value})), ctypes.byref(info))
    assert rc == code
    assert msg in lib.pdp_last_error()


def test_pair_table_modes_plan(lib):
    """l0 = 0 (LinfSampler / NoOpSampler), max_contributions and
    rows_are_units resolve to the pair-table algorithm; their exclusions
    mirror AggregateParams (aggregate_params.py:344-369)."""
    info = N.BoundPlanInfo()
    for kw in (dict(l0=0), dict(l0=0, linf=0), dict(l0=0, linf=0, max_contributions=5),
               dict(l0=0, linf=0, rows_are_units=1)):
        assert lib.pdp_bound_plan(ctypes.byref(_cfg(**kw)), ctypes.byref(info)) == 0, kw
        assert info.algorithm == N.ALGO_PAIR_TABLE
        ws = ctypes.c_uint64(0)
        assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(**kw)), ctypes.byref(ws)) == 0
        assert ws.value > 0
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(l0=2, linf=0, max_contributions=5)), ctypes.byref(info)) == -1
    assert b"max_contributions" in lib.pdp_last_error()
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(l0=0, linf=1, rows_are_units=1)), ctypes.byref(info)) == -1
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(l0=0, algorithm=N.ALGO_BUCKETED)), ctypes.byref(info)) == -4
    # PAIR_TABLE with cross-partition sampling: L0 over the table's distinct pairs
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(l0=2, algorithm=N.ALGO_PAIR_TABLE)), ctypes.byref(info)) == 0
    assert info.algorithm == N.ALGO_PAIR_TABLE
    # bounds above 256 (l0, linf, max_contributions) resolve to the pair table
    for kw in (dict(l0=257), dict(l0=2, linf=300), dict(l0=100_000, linf=100_000),
               dict(l0=0, linf=0, max_contributions=10_000), dict(l0=2**31 - 1, linf=1)):
        assert lib.pdp_bound_plan(ctypes.byref(_cfg(**kw)), ctypes.byref(info)) == 0, kw
        assert info.algorithm == N.ALGO_PAIR_TABLE, kw
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(l0=300, algorithm=N.ALGO_BUCKETED)), ctypes.byref(info)) == -4
    # rows_are_units needs no privacy-id column
    cfg = _cfg(n_rows=10, l0=0, linf=0, rows_are_units=1)
    need = ctypes.c_uint64(0)
    lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(need))
    rc = lib.pdp_bound_contributions(ctypes.byref(cfg), None, None, None, None, ctypes.c_void_p(256),
                                     need.value, None)
    assert rc == -1 and b"key columns" in lib.pdp_last_error()


def test_sum_int_needs_int_values(lib):
    info = N.BoundPlanInfo()
    rc = lib.pdp_bound_plan(ctypes.byref(_cfg(flags=N.ACC_SUM | N.SUM_INT)), ctypes.byref(info))
    assert rc == -1 and b"PDP_SUM_INT" in lib.pdp_last_error()


def test_null_arguments_are_rejected_before_device_work(lib):
    cfg = _cfg(n_rows=10)
    assert lib.pdp_bound_plan(ctypes.byref(cfg), None) == -1
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), None) == -1
    assert lib.pdp_bound_plan(None, ctypes.byref(N.BoundPlanInfo())) == -1
    # workspace too small: refused before any launch
    rc = lib.pdp_bound_contributions(ctypes.byref(cfg), None, None, None, None, None, 0, None)
    assert rc == -3
    # key columns missing with a big enough (fake, never dereferenced) workspace pointer
    need = ctypes.c_uint64(0)
    lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(need))
    rc = lib.pdp_bound_contributions(ctypes.byref(cfg), None, None, None, None, ctypes.c_void_p(256),
                                     need.value, None)
    assert rc == -1 and b"key columns" in lib.pdp_last_error()


def test_dataset_histograms_arguments(lib):
    need = ctypes.c_uint64(0)
    assert lib.pdp_dataset_histograms_workspace_bytes(1000, 100, 10, ctypes.byref(need)) == 0
    # pair table (1.5 slots of 32 bytes per row) + per-pid / per-partition arrays
    assert need.value >= 1500 * 32 + 100 * 8 + 10 * 16
    assert lib.pdp_dataset_histograms_workspace_bytes(-1, 100, 10, ctypes.byref(need)) == -1
    assert lib.pdp_dataset_histograms_workspace_bytes(10, 100, 10, None) == -1
    out = N.HistogramBins()  # every output NULL: refused before device work
    rc = lib.pdp_dataset_histograms(None, None, None, N.VALUE_F64, 10, 100, 10, ctypes.byref(out), None, 0, None)
    assert rc == -1 and b"output" in lib.pdp_last_error()
    fake = N.HistogramBins(*([256] * 8))  # never dereferenced: the shape checks fail first
    rc = lib.pdp_dataset_histograms(None, None, None, N.VALUE_F64, 1 << 31, 100, 10, ctypes.byref(fake), None, 0,
                                    None)
    assert rc == -4
    rc = lib.pdp_dataset_histograms(None, None, None, N.VALUE_F64, 10, 1 << 40, 1 << 30, ctypes.byref(fake),
                                    None, 0, None)
    assert rc == -4 and b"63 bits" in lib.pdp_last_error()
    rc = lib.pdp_dataset_histograms(None, None, None, N.VALUE_F64, 10, 100, 10, ctypes.byref(fake), None, 0, None)
    assert rc == -1 and b"workspace" in lib.pdp_last_error()


def test_debug_corrupt_flag_needs_test_hooks(lib, monkeypatch):
    """PDP_DEBUG_CORRUPT_RECORDS (it overwrites level-2 records on purpose)
    is rejected unless PIPELINEDP_AMD_TEST_HOOKS=1."""
    nbytes = ctypes.c_uint64(0)
    cfg = _cfg(flags=N.ACC_NSUM | N.DEBUG_CORRUPT_RECORDS)
    monkeypatch.delenv("PIPELINEDP_AMD_TEST_HOOKS", raising=False)
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)) == -1
    assert b"test hook" in lib.pdp_last_error()
    monkeypatch.setenv("PIPELINEDP_AMD_TEST_HOOKS", "1")
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)) == 0


def test_sieve_threads_plan(lib):
    """sieve_threads: 0 (auto) and 1024 resolve to 1,024-thread level-1
    workgroups, 512 to two per CU when their LDS fits; other values fail."""
    info = N.BoundPlanInfo()
    c3 = dict(n_rows=1_000_000_000, n_privacy_ids=10_000_000, n_partitions=1_000_000, l0=2, linf=1)
    for want, got in ((0, 1024), (1024, 1024), (512, 512)):
        assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve_threads=want)), ctypes.byref(info)) == 0
        assert info.sieve > 0 and info.sieve_threads == got
    assert lib.pdp_bound_plan(ctypes.byref(_cfg(**c3, sieve=-1)), ctypes.byref(info)) == 0
    assert info.sieve_threads == 0
    nbytes = ctypes.c_uint64(0)
    assert lib.pdp_bound_workspace_bytes(ctypes.byref(_cfg(**c3, sieve_threads=256)), ctypes.byref(nbytes)) == -1
