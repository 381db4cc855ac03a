"""CPU checks of the specialised-kernel tier (mythril_amd/jit.py, csrc/mw_jit.h).

The generated source is compiled twice: for gfx950 (code-object checks: it
builds, carries the program signature and both kernels, and the straight-line
body does not spill to scratch) and for x86 (a host build of the very same
body), whose verdicts and traced node values are compared with the oracle
and with the interpreter's host build on generated candidates — pools of edge
values (0, 1, 2^w-1, 2^(w-1), w, ...) mixed with Philox draws.  The device
parity tests are tests/test_gpu_jit.py.
"""
import ctypes
import random
import re
import subprocess

import numpy as np
import pytest

from mythril_amd import jit
from mythril_amd.compiler import LeafSpec, compile_program
from mythril_amd.ir import BOOL, topo
from mythril_amd.runtime import unpack_trace
from oracle.dag_eval import eval_nodes
from tests.helpers import RandDag, emu_eval, oracle_models

LLVM = "/opt/rocm/lib/llvm/bin"


def edge_pool(w):
    m = (1 << w) - 1
    vals = [0, 1, 2, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, (1 << (w - 1)) + 1, w, w - 1, w + 1, 3]
    return [v & m for v in vals] + [None] * 4


def edge_specs(dag):
    specs = {}
    for v in dag.vars + dag.bvars:
        w = 1 if v.width == BOOL else v.width
        specs[v.name] = LeafSpec(v.name, w, pool=edge_pool(w) if w > 1 else [0, 1], hashed=True)
    return specs


def host_run(lib, name, p, seed, begin, n, early=False):
    f = getattr(lib, name + "_host")
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                  ctypes.c_void_p, ctypes.c_void_p]
    pool = np.ascontiguousarray(p.pool, dtype=np.uint32)
    v = np.zeros(n, dtype=np.uint32)
    t = np.zeros(max(p.n_trace_rows, 1) * n, dtype=np.uint32)
    assert f(pool.ctypes.data, seed, begin, n, 1 if early else 0, v.ctypes.data, t.ctypes.data) == 0
    return v, t.reshape(max(p.n_trace_rows, 1), n)


def _random_programs(nprog, base_seed):
    out = []
    for k in range(nprog):
        rng = random.Random(base_seed + k)
        dag = RandDag(base_seed + k)
        conj = [dag.boolean(4) for _ in range(3)]
        extra = [dag.bv(rng.choice(dag.widths), 4) for _ in range(4)]
        nodes = [n for n in topo(conj + extra) if not n.is_array]
        p = compile_program(conj, trace=nodes, leaf_specs=edge_specs(dag))
        out.append((dag, conj, extra, nodes, p))
    return out


@pytest.fixture(scope="module")
def host_lib():
    progs = _random_programs(24, 7000)
    path, names = jit.compile_host([p for *_, p in progs])
    return ctypes.CDLL(str(path)), progs, names


def test_host_build_matches_oracle_and_interpreter(host_lib):
    lib, progs, names = host_lib
    seed, begin, n = 0x5EED0007, 1 << 33, 48
    for (dag, conj, extra, nodes, p), name in zip(progs, names):
        v, tr = host_run(lib, name, p, seed, begin, n)
        models = oracle_models(p, seed, begin, n)
        for j, m in enumerate(models):
            vals = eval_nodes(conj + extra, m)
            assert v[j] == int(all(vals[c.id] for c in conj)), f"{name} verdict {j}"
        for node in nodes:
            got = unpack_trace(p, tr, node)
            for j, m in enumerate(models):
                exp = eval_nodes([node], m)[node.id]
                assert got[j] == exp, f"{name} {node!r}[{j}]: {got[j]:#x} != {exp:#x}"
        iv, _ = emu_eval(p, None, n, seed=seed, begin=begin)
        assert list(iv) == list(v), f"{name}: interpreter verdicts differ"


def test_host_build_early_exit_agrees(host_lib):
    lib, progs, names = host_lib
    for (_, _, _, _, p), name in zip(progs, names):
        a, _ = host_run(lib, name, p, 3, 0, 64, early=False)
        b, _ = host_run(lib, name, p, 3, 0, 64, early=True)
        assert list(a) == list(b)


def test_signature_matches_library_definition():
    # the C side (mw_kernels.hip prog_signature) hashes the same words FNV-1a 64
    rng = random.Random(2)
    dag = RandDag(2)
    p = compile_program([dag.boolean(3)])
    h = 0xCBF29CE484222325
    for arr in (p.code, p.consts, p.leaves, p.pool):
        for wd in np.asarray(arr, dtype=np.uint32).tolist():
            for b in range(4):
                h ^= (wd >> (8 * b)) & 0xFF
                h = (h * 0x100000001B3) & ((1 << 64) - 1)
    assert jit.signature(p) == h
    assert jit.kernel_name(p) == f"mwj_{h:016x}"


def test_identical_programs_share_one_kernel():
    # two queries of one launch group that compile to the same program
    # (config_bench's LASER groups have such pairs) must not define it twice
    p = compile_program([RandDag(5).boolean(3)])
    q = compile_program([RandDag(5).boolean(3)])
    assert jit.kernel_name(p) == jit.kernel_name(q)
    src = jit.generate([p, q], [jit.kernel_name(p)] * 2)
    assert src.count("MW_JIT_SIG(") == 1
    assert src.count(f"MW_JIT_KERNEL({jit.kernel_name(p)}, _x") == 1


def _unbundle(hsaco_bytes, tmp_path):
    src = tmp_path / "k.hsaco"
    src.write_bytes(hsaco_bytes)
    elf = tmp_path / "k.elf"
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={src}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], check=True)
    return elf


def test_device_code_object(tmp_path):
    from tests.test_gpu_jit import small_planted
    s = small_planted(n_nodes=400, n_conj=8)
    p = compile_program(s.conjuncts)
    image, names, _ = jit.compile_device([p])
    elf = _unbundle(image, tmp_path)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", "--syms", str(elf)], capture_output=True,
                           text=True).stdout
    name = names[0]
    for sym in (name + "_x", name + "_e", name + "_sig"):
        assert sym in notes, sym
    # 2 waves/SIMD: at most 256 VGPRs, and the straight-line body stays in registers
    vg = [int(x) for x in re.findall(r"\.vgpr_count:\s+(\d+)", notes)]
    sp = [int(x) for x in re.findall(r"\.vgpr_spill_count:\s+(\d+)", notes)]
    assert vg and max(vg) <= 256
    assert sp and max(sp) <= 8, f"VGPR spills {sp}"


def test_host_build_division_rare_paths():
    from tests.helpers import division_check_programs
    progs = division_check_programs()
    path, names = jit.compile_host(progs)
    lib = ctypes.CDLL(str(path))
    for p, name in zip(progs, names):
        v, _ = host_run(lib, name, p, 1, 0, 256)
        assert int(v.sum()) == 256, name


def test_host_build_lds_leaves_match_oracle():
    """Leaves kept in LDS (reloaded at every use) give the same values."""
    progs = _random_programs(6, 7300)
    path, names = jit.compile_host([p for *_, p in progs], lds_leaves=3)
    src = jit.generate([p for *_, p in progs], names, "", lds_leaves=3)
    assert "lds_put8" in src and "lds_get8" in src
    lib = ctypes.CDLL(str(path))
    seed, begin, n = 0x5EED0008, 77, 40
    for (dag, conj, extra, nodes, p), name in zip(progs, names):
        v, tr = host_run(lib, name, p, seed, begin, n)
        models = oracle_models(p, seed, begin, n)
        for j, m in enumerate(models):
            vals = eval_nodes(conj + extra, m)
            assert v[j] == int(all(vals[c.id] for c in conj)), f"{name} verdict {j}"
            for node in nodes:
                assert unpack_trace(p, tr, node)[j] == vals[node.id], f"{name} {node!r}[{j}]"


def test_host_build_parts_and_to_whole_program():
    """A program split into parts (jit.split_ssa) is the AND of its parts."""
    from tests.test_gpu_jit import small_planted
    s = small_planted(n_nodes=400, n_conj=8, density_log2=6)
    p = compile_program(s.conjuncts)
    segs = jit.split_ssa(p, part_weight=3000)
    assert len(segs) >= 3
    path, names = jit.compile_host([p], part_weight=3000)
    lib = ctypes.CDLL(str(path))
    n, begin = 512, s.witness_index - 300
    acc = np.ones(n, dtype=np.uint32)
    for name in names:
        v, _ = host_run(lib, name, p, s.seed, begin, n)
        acc &= v
    whole, _ = emu_eval(p, None, n, seed=s.seed, begin=begin)
    assert np.array_equal(acc, whole)
    assert acc[300] == 1  # the planted witness


@pytest.mark.parametrize("ahead", [0, 8, 32])
def test_lds_reloads_ahead_of_use(monkeypatch, ahead):
    """jit.LDS_AHEAD: a leaf's LDS reload moves up to `ahead` body lines
    before its use, never above the leaf's own store; the host build with
    the reloads moved still gives the oracle's verdicts."""
    import re
    monkeypatch.setattr(jit, "LDS_AHEAD", ahead)
    progs = _random_programs(4, 7400)
    src = jit.generate([p for *_, p in progs], [f"t{k}" for k in range(len(progs))], "", lds_leaves=3)
    bodies = src.split("template <bool EARLY>")[1:]     # names restart in every program's body
    assert len(bodies) == len(progs)
    for text in bodies:
        body = text.splitlines()
        decl, put = {}, {}
        for i, ln in enumerate(body):
            for m in re.finditer(r"u32 (L\d+)\[8\]; jit::lds_get8\((\d+)u", ln):
                decl[m.group(1)] = (i, int(m.group(2)))
            for m in re.finditer(r"jit::lds_put8\((\d+)u", ln):
                put.setdefault(int(m.group(1)), []).append(i)
        assert decl
        for i, ln in enumerate(body):
            for m in re.finditer(r"\b(L\d+)\b(?!\[8\])", ln):
                at, slot = decl[m.group(1)]
                assert at <= i, (m.group(1), at, i)
                # the reload follows a store of its slot
                assert any(p < at for p in put.get(slot, [])), (m.group(1), slot)
    path, names = jit.compile_host([p for *_, p in progs], lds_leaves=3)
    lib = ctypes.CDLL(str(path))
    seed, begin, n = 0x5EED000A, 91, 24
    for (dag, conj, extra, nodes, p), name in zip(progs, names):
        v, _ = host_run(lib, name, p, seed, begin, n)
        for j, m in enumerate(oracle_models(p, seed, begin, n)):
            vals = eval_nodes(conj, m)
            assert v[j] == int(all(vals[c.id] for c in conj)), f"{name} verdict {j}"
