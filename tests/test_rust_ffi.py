"""The Rust binding (rust/ggrs-mi355x/src/ffi.rs) against the C header (include/ggrs_amd.h): every
function the header declares is declared in Rust with the same parameter count and types, every
ABI struct has the same fields in the same order with the same types, every GGRS_* constant has
the same value.  No Rust toolchain in this image: the check parses both files.  CPU only."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ggrs_amd.h")
FFI = os.path.join(ROOT, "rust", "ggrs-mi355x", "src", "ffi.rs")

C_BASE = {"int": "i32", "int32_t": "i32", "int64_t": "i64", "uint8_t": "u8", "uint16_t": "u16",
          "uint32_t": "u32", "uint64_t": "u64", "float": "f32", "char": "c_char", "void": "c_void"}


def strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def c_type(t):
    """'const uint8_t*' -> ('*const', 'u8'); 'ggrs_engine_t**' -> ('*mut*mut', 'ggrs_engine_t')."""
    t = t.strip()
    stars = t.count("*")
    is_const = t.startswith("const ")
    base = t.replace("const ", "").replace("*", "").strip()
    base = C_BASE.get(base, base)
    if stars == 0:
        return ("", base)
    ptr = ("*const" if is_const else "*mut") + "*mut" * (stars - 1)
    return (ptr, base)


def rust_type(t):
    t = t.strip()
    ptr = ""
    while t.startswith("*"):
        m = re.match(r"\*(const|mut)\s+", t)
        ptr += "*" + m.group(1)
        t = t[m.end():]
    return (ptr, t.strip())


def split_params(p):
    p = " ".join(p.split())
    if p in ("", "void"):
        return []
    return [x.strip() for x in p.split(",") if x.strip()]


def header_functions():
    src = strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"^\s*((?:const\s+)?[A-Za-z_0-9]+\s*\*?)\s*(ggrs_\w+)\s*\(([^)]*)\)\s*;", src, re.M):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = []
        for p in split_params(params):
            mm = re.match(r"(.*?)([A-Za-z_]\w*)$", p)
            ps.append(c_type(mm.group(1)))
        out[name] = (c_type(ret), ps)
    return out


def rust_functions():
    src = open(FFI).read()
    body = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (ggrs_\w+)\(([^)]*)\)\s*(?:->\s*([^;]+))?;", body, re.S):
        name, params, ret = m.group(1), m.group(2), (m.group(3) or "()").strip()
        ps = [rust_type(p.split(":", 1)[1]) for p in split_params(params)]
        out[name] = (rust_type(ret), ps)
    return out


def header_structs():
    src = strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct \w+ \{(.*?)\} (\w+);", src, re.S):
        fields = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            mm = re.match(r"(.*?)([A-Za-z_]\w*)$", decl)
            fields.append((mm.group(2), c_type(mm.group(1))))
        out[m.group(2)] = fields
    return out


def rust_structs():
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\][^\n]*\n(?:#\[derive[^\n]*\n)?pub struct (\w+) \{(.*?)\n\}", src, re.S):
        fields = []
        for line in m.group(2).split(","):
            line = line.strip()
            if not line.startswith("pub "):
                continue
            name, ty = line[4:].split(":", 1)
            fields.append((name.strip(), rust_type(ty)))
        out[m.group(1)] = fields
    return out


def test_every_header_function_is_bound_with_the_same_signature():
    h, r = header_functions(), rust_functions()
    assert len(h) > 80
    missing = sorted(set(h) - set(r))
    assert not missing, f"not declared in ffi.rs: {missing}"
    extra = sorted(set(r) - set(h))
    assert not extra, f"ffi.rs declares functions the header does not: {extra}"
    for name, (ret, ps) in h.items():
        rret, rps = r[name]
        assert rret == ret, (name, ret, rret)
        assert len(rps) == len(ps), (name, len(ps), len(rps))
        for i, (a, b) in enumerate(zip(ps, rps)):
            assert a == b, (name, i, a, b)


def test_every_abi_struct_matches_field_by_field():
    h, r = header_structs(), rust_structs()
    assert {"ggrs_config_t", "ggrs_request_t", "ggrs_lane_batch_t", "ggrs_branch_config_t",
            "ggrs_particle_config_t", "ggrs_p2p_config_t"} <= set(h)
    for name, fields in h.items():
        assert name in r, f"struct {name} missing from ffi.rs"
        assert r[name] == fields, name


def test_constants_match():
    src = strip_c_comments(open(HEADER).read())
    consts = {m.group(1): int(m.group(2).strip("()")) for m in
              re.finditer(r"#define (GGRS_\w+)\s+(\(?-?\d+\)?)", src)}
    rs = {m.group(1): int(m.group(2)) for m in
          re.finditer(r"pub const (GGRS_\w+): \w+ = (-?\d+);", open(FFI).read())}
    assert len(consts) > 30
    for k, v in consts.items():
        assert k in rs, f"{k} missing from ffi.rs"
        assert rs[k] == v, k


def test_build_rs_compiles_every_unit_with_build_py_flags():
    """build.rs hands hipcc the same translation units as ggrs_amd/build.py (a unit missing there
    leaves its symbols undefined in the crate's library), with the same common flags and the same
    per-unit flags (max-ilp on the step-kernel units), so the crate links the library bench.py
    measures."""
    from ggrs_amd import build
    src = open(os.path.join(ROOT, "rust", "ggrs-mi355x", "build.rs")).read()

    def str_list(name):
        m = re.search(r"const %s: &\[&str\] = &\[(.*?)\];" % name, src, re.S)
        assert m, name
        return re.findall(r'"([^"]*)"', m.group(1))

    assert str_list("FLAGS") == build.FLAGS
    lists = {"ILP": str_list("ILP"), "NONE": str_list("NONE")}
    assert lists["ILP"] == build.ILP and lists["NONE"] == []
    m = re.search(r"const UNITS: &\[\(&str, &\[&str\]\)\] = &\[(.*?)\];", src, re.S)
    assert m
    units = re.findall(r'\("(\w+\.(?:hip|cpp))",\s*(\w+)\)', m.group(1))
    assert [u for u, _ in units] == list(build.UNITS)
    for unit, flags in units:
        assert lists[flags] == build.UNIT_FLAGS.get(unit, []), unit
