"""CPU: the C-ABI library loads, exports every symbol include/polaroid_gpu.h
declares, its struct layouts match the ctypes mirror, and host-side
validation (program type-checking, argument checks) errors without a GPU."""

import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "polaroid_gpu.h")


@pytest.fixture(scope="module")
def N():
    from polaroid_amd import _native

    if not os.path.exists(_native.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "polaroid_amd", "csrc")], check=True)
    _native.lib()
    return _native


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(plgpu_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound(N):
    decl = declared_functions()
    assert len(decl) >= 15
    lib = C.CDLL(N.LIB_PATH)
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in include/polaroid_gpu.h but not exported"
        assert name in N.SIGNATURES, f"{name} not bound in polaroid_amd/_native.py"
    assert sorted(N.SIGNATURES) == decl


def test_struct_layouts_match_header(N):
    probe = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "polaroid_gpu.h"
    int main(void) {
      printf("%zu %zu %zu %zu %zu\n", sizeof(plgpu_column), offsetof(plgpu_column, values),
             offsetof(plgpu_column, release), sizeof(plgpu_instr), offsetof(plgpu_instr, imm));
      printf("%zu %zu %zu\n", sizeof(plgpu_agg), sizeof(plgpu_groupby_info),
             offsetof(plgpu_groupby_info, main_kernel_ms));
      return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "p.c"), os.path.join(d, "p")
        open(src, "w").write(probe)
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    got = [int(x) for x in out]
    exp = [C.sizeof(N.Column), N.Column.values.offset, N.Column.release.offset, C.sizeof(N.Instr),
           N.Instr.imm.offset, C.sizeof(N.Agg), C.sizeof(N.GroupByInfo), N.GroupByInfo.main_kernel_ms.offset]
    assert got == exp


def test_abi_version(N):
    assert N.lib().plgpu_abi_version() == 1


def _instrs(N, prog):
    arr = (N.Instr * len(prog))()
    for i, (op, arg, imm) in enumerate(prog):
        arr[i].op, arr[i].arg = op, arg
        if op == N.OP["LIT_F64"]:
            arr[i].imm.f64 = imm
        else:
            arr[i].imm.i64 = imm
    return arr


def _host_col(N, dtype, n):
    c = N.Column()
    c.dtype, c.length = dtype, n
    c.values = 0x1000  # never dereferenced: validation fails before any device work
    return c


@pytest.mark.parametrize(
    "prog, code",
    [
        ([("AND", 0, 0)], "ERR_INVALID"),                                   # stack underflow
        ([("COL", 0, 0), ("LIT_BOOL", 0, 1), ("ADD", 0, 0)], "ERR_INVALID"),  # bool arithmetic
        ([("COL", 0, 0), ("NOT", 0, 0)], "ERR_SCHEMA"),                     # not on f64
        ([("COL", 0, 0), ("COL", 1, 0), ("AND", 0, 0)], "ERR_SCHEMA"),      # and on numerics
        ([("COL", 5, 0)], "ERR_INVALID"),                                   # bad column index
        ([("COL", 1, 0), ("IS_NAN", 0, 0)], "ERR_INVALID"),                 # is_nan on int
        ([("COL", 0, 0), ("COL", 0, 0)], "ERR_INVALID"),                    # two results
    ],
)
def test_program_type_errors_without_gpu(N, prog, code):
    cols = (N.Column * 2)(_host_col(N, N.F64, 4), _host_col(N, N.I64, 4))
    p = _instrs(N, [(N.OP[o], a, i) for o, a, i in prog])
    out = N.Column()
    rc = N.lib().plgpu_eval(cols, 2, p, len(prog), C.byref(out), None)
    assert rc == getattr(N, code), N.lib().plgpu_last_error()
    assert N.lib().plgpu_last_error()


def test_filter_predicate_must_be_boolean_without_gpu(N):
    cols = (N.Column * 1)(_host_col(N, N.F64, 4))
    p = _instrs(N, [(N.OP["COL"], 0, 0), (N.OP["LIT_F64"], 0, 1.0), (N.OP["ADD"], 0, 0)])
    out = (N.Column * 1)()
    n = C.c_int64()
    rc = N.lib().plgpu_filter_expr(cols, 1, p, 3, out, C.byref(n), None)
    assert rc == N.ERR_SCHEMA
    assert "must be of type `Boolean`" in N.lib().plgpu_last_error().decode()


def test_group_by_argument_checks_without_gpu(N):
    key = _host_col(N, N.F64, 4)
    cols = (N.Column * 1)(_host_col(N, N.F64, 4))
    aggs = (N.Agg * 1)()
    aggs[0].kind, aggs[0].col = N.AGG["sum"], 0
    ok, outs = N.Column(), (N.Column * 1)()
    rc = N.lib().plgpu_group_by_agg(C.byref(key), cols, 1, None, 0, aggs, 1, 0, C.byref(ok), outs, None, None)
    assert rc == N.ERR_SCHEMA  # key must be Int64/Int32
    key = _host_col(N, N.I64, 4)
    cols = (N.Column * 1)(_host_col(N, N.F64, 5))
    rc = N.lib().plgpu_group_by_agg(C.byref(key), cols, 1, None, 0, aggs, 1, 0, C.byref(ok), outs, None, None)
    assert rc == N.ERR_SHAPE


def _header_decls():
    """{name: number of parameters} of every function include/polaroid_gpu.h
    declares, and {struct: [field names]} of its typedef'd structs."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    funcs = {}
    for m in re.finditer(r"\b(plgpu_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        args = m.group(2).strip()
        funcs[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    structs = {}
    for m in re.finditer(r"typedef struct (\w+)\s*\{(.*?)\}\s*\w+\s*;", text, flags=re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = line.strip()
            if not line:
                continue
            fp = re.search(r"\(\s*\*\s*(\w+)\s*\)", line)  # a function-pointer field
            fm = fp or re.search(r"(\w+)\s*(\[[^\]]*\])?\s*$", line)
            if fm:
                fields.append(fm.group(1))
        structs[m.group(1)] = fields
    return funcs, structs


def _rust_decls():
    """The same from INTEGRATION.md's Rust `extern "C"` block and structs."""
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blk = md[md.index('extern "C" {'):]
    blk = blk[:blk.index("\n}\n")]
    blk = re.sub(r"//[^\n]*", "", blk)
    funcs = {}
    for m in re.finditer(r"pub fn (plgpu_\w+)\((.*?)\)\s*(->\s*[\w\s\*]+)?;", blk, flags=re.S):
        args = m.group(2).strip()
        funcs[m.group(1)] = 0 if not args else args.count(":")
    structs = {}
    code = md[:md.index('extern "C" {')]
    for m in re.finditer(r"pub struct (\w+)\s*\{(.*?)\}", code, flags=re.S):
        body = re.sub(r"//[^\n]*", "", m.group(2))
        structs[m.group(1)] = re.findall(r"pub (\w+)\s*:", body)
    return funcs, structs


def test_integration_rust_bindings_match_header():
    """INTEGRATION.md's Rust extern block binds exactly the header's
    functions with the header's parameter counts, and its structs list the
    header's fields in the header's order (round-5 verdict: the doc had
    drifted -- a renamed field, twelve unbound exports)."""
    hf, hs = _header_decls()
    rf, rs = _rust_decls()
    assert sorted(hf) == sorted(rf), (sorted(set(hf) - set(rf)), sorted(set(rf) - set(hf)))
    bad = {n: (hf[n], rf[n]) for n in hf if hf[n] != rf[n]}
    assert not bad, f"parameter counts differ (header, Rust): {bad}"
    for c_name, r_name in (("plgpu_groupby_info", "PlgpuGroupByInfo"), ("plgpu_column", "PlgpuColumn")):
        assert hs[c_name] == rs[r_name], (c_name, hs[c_name], rs[r_name])


def test_documented_options_exist(N):
    """Every option name the header documents under plgpu_set_option is one
    the library knows (set, read back, restored) -- no GPU needed; an
    undocumented name is PLGPU_ERR_INVALID."""
    import re

    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "polaroid_gpu.h")).read()
    i = hdr.index("int plgpu_set_option(")
    block = hdr[hdr.rindex("/*", 0, i):i]
    names = sorted(set(re.findall(r'^\s*\*\s+"([a-z0-9_]+)"', block, re.M)))
    assert len(names) >= 20, names
    for name in names:
        prev = N.set_option(name, 0)
        assert N.set_option(name, prev) == 0, name
    v = C.c_int64(0)
    assert N.lib().plgpu_get_option(b"no_such_option", C.byref(v)) == N.ERR_INVALID
