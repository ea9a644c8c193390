"""The Rust binding's declarations (bindings/rust/src/crypto/mi355x/ffi.rs, UNCOMPILED: no cargo here)
against the C-ABI header include/sda_engine.h: every C function is declared in the `extern "C"` block with
the same argument names, count, order, integer widths and const-ness, and the two scheme structs match
field for field.  Text-level: the Rust is parsed, not compiled."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sda_engine.h")
FFI = os.path.join(ROOT, "bindings", "rust", "src", "crypto", "mi355x", "ffi.rs")

# C type (normalised) -> Rust type
_SCALAR = {"int64_t": "i64", "uint64_t": "u64", "int32_t": "i32", "uint32_t": "u32", "uint8_t": "u8",
           "int": "c_int", "void": "c_void", "char": "c_char", "sda_engine": "SdaEngine",
           "sda_sharing_scheme": "SdaSharingScheme", "sda_masking_scheme": "SdaMaskingScheme",
           "sda_status": "SdaStatus"}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", re.sub(r"//[^\n]*", " ", s, flags=re.S), flags=re.S)


def _c_type_to_rust(ctype):
    """'const int64_t* const*' -> '*const *const i64' (C pointer levels read right to left)."""
    t = ctype.replace("*", " * ").split()
    # split into the base (with its const) and pointer levels, each with the const that FOLLOWS it
    base_const = False
    base = None
    levels = []            # per '*': is the pointee at that level const?
    pending_const = False
    for tok in t:
        if tok == "const":
            pending_const = True
        elif tok == "*":
            levels.append(pending_const if levels else (base_const or pending_const))
            pending_const = False
        else:
            base = tok
            base_const, pending_const = pending_const, False
    rust = _SCALAR[base]
    # the innermost '*' points at the base; each next '*' points at the previous pointer
    for i, const in enumerate(levels):
        rust = ("*const " if const else "*mut ") + rust
    return rust


def _c_functions():
    src = _strip_c_comments(open(HEADER).read())
    body = src[src.index('extern "C" {') + len('extern "C" {'):]
    funcs = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(sda_\w+)\s*\(([^)]*)\)\s*;", body):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                pm = re.match(r"(.*?)(\w+)$", a)
                ctype, pname = pm.group(1).strip(), pm.group(2)
                params.append((pname, _c_type_to_rust(ctype)))
        funcs[name] = (_c_type_to_rust(ret), params)
    return funcs


def _rust_functions():
    src = re.sub(r"//[^\n]*", " ", open(FFI).read())
    block = src[src.index('extern "C" {'):]
    funcs = {}
    for m in re.finditer(r"pub fn (sda_\w+)\s*\(([^)]*)\)\s*(->\s*([^;]+))?;", block):
        name, args, ret = m.group(1), m.group(2), (m.group(4) or "()").strip()
        params = []
        for a in [x for x in args.split(",") if x.strip()]:
            pname, ptype = a.split(":", 1)
            params.append((pname.strip(), " ".join(ptype.split())))
        funcs[name] = (ret, params)
    return funcs


def _norm_ret(r):
    return {"c_void": "()", "SdaStatus": "SdaStatus"}.get(r, r)


def test_every_c_function_is_declared_identically():
    c, rs = _c_functions(), _rust_functions()
    assert len(c) >= 40, sorted(c)
    assert sorted(c) == sorted(rs), (set(c) ^ set(rs))
    for name, (cret, cparams) in c.items():
        rret, rparams = rs[name]
        assert _norm_ret(cret) == rret, (name, cret, rret)
        assert len(cparams) == len(rparams), (name, cparams, rparams)
        for (cn, ct), (rn, rt) in zip(cparams, rparams):
            assert cn == rn, (name, cn, rn)
            assert ct == rt, (name, cn, ct, rt)


def _c_struct(name):
    src = _strip_c_comments(open(HEADER).read())
    m = re.search(r"typedef struct \{([^}]*)\}\s*" + name + ";", src)
    return [(f.split()[-1], _SCALAR[f.split()[0]]) for f in m.group(1).split(";") if f.strip()]


def _rust_struct(name):
    src = open(FFI).read()
    m = re.search(r"pub struct " + name + r" \{([^}]*)\}", src)
    out = []
    for f in m.group(1).split(","):
        f = f.strip()
        if f:
            fname, ftype = f.replace("pub ", "").split(":")
            out.append((fname.strip(), ftype.strip()))
    return out


def test_scheme_structs_match_field_for_field():
    assert _c_struct("sda_sharing_scheme") == _rust_struct("SdaSharingScheme")
    assert _c_struct("sda_masking_scheme") == _rust_struct("SdaMaskingScheme")


def test_status_codes_match():
    src = _strip_c_comments(open(HEADER).read())
    enum = re.search(r"typedef enum \{(.*?)\} sda_status;", src, flags=re.S).group(1)
    c = {k: int(v) for k, v in re.findall(r"(SDA_\w+)\s*=\s*(\d+)", enum)}
    rs = {k: int(v) for k, v in re.findall(r"pub const (SDA_\w+): SdaStatus = (\d+);", open(FFI).read())}
    assert c == rs


def test_type_mapping_reads_pointer_levels():
    assert _c_type_to_rust("const int64_t* const*") == "*const *const i64"
    assert _c_type_to_rust("sda_engine**") == "*mut *mut SdaEngine"
    assert _c_type_to_rust("const uint8_t* const*") == "*const *const u8"
    assert _c_type_to_rust("void*") == "*mut c_void"
    assert _c_type_to_rust("const void*") == "*const c_void"
