"""CPU checks of the Rust binding crate rust/dips-hip against the C ABI it
binds (no Rust toolchain in this image, so the crate is checked as source):

* every #[repr(C)] struct of src/ffi.rs has the header struct's fields, in
  order, with the mapped types;
* every function include/dips_hip.h declares is declared in the extern block
  with the same parameter and return types (and nothing else is);
* the sizes / offsets the Rust `const` asserts pin equal the ones gcc
  computes for the C structs, and the header's own DIPS_LAYOUT_ASSERTs hold
  under C99 and C++17.

Reference items replaced: dips/src/gpu/mod.rs:59-65, :170, :306 and
dips/src/lib.rs:23, :32-61 (ComputeState, CallbackFunction, the filter codes)."""
import os
import re
import subprocess


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dips_hip.h")
CRATE = os.path.join(ROOT, "rust", "dips-hip")
FFI = os.path.join(CRATE, "src", "ffi.rs")

STRUCTS = {"dips_params": "DipsParams", "dips_series_entry": "DipsSeriesEntry", "dips_alt_params": "DipsAltParams"}
BASE = {"uint8_t": "u8", "uint16_t": "u16", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64",
        "float": "f32", "double": "f64", "size_t": "usize", "int": "c_int", "void": "c_void", "char": "c_char",
        "dips_status": "DipsStatus", "dips_handle": "DipsHandle", "dips_alt_handle": "DipsAltHandle",
        "dips_comm": "DipsComm", "dips_comm_ops": "DipsCommOps",
        **STRUCTS}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_to_rust(decl):
    """'const uint8_t *frame' -> '*const u8' (the name dropped)."""
    decl = decl.strip()
    stars = decl.count("*")
    toks = decl.replace("*", " ").split()
    const = "const" in toks
    toks = [t for t in toks if t != "const"]
    base = BASE[toks[0]]
    if stars == 0:
        return base
    inner = base
    for level in range(stars):
        # the innermost pointer carries the const of the pointee
        inner = f"*{'const' if const and level == 0 else 'mut'} {inner}"
    return inner


def _c_ret(ret):
    ret = ret.strip()
    if ret == "void":
        return None
    return _c_to_rust(ret)


def header_structs():
    src = _strip_c_comments(open(HEADER).read())
    out = {}
    for name in STRUCTS:
        m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S)
        assert m, name
        fields = []
        for line in m.group(1).split(";"):
            line = line.strip()
            if line:
                *ty, field = line.split()
                fields.append((field, BASE[" ".join(ty)]))
        out[name] = fields
    return out


def header_functions():
    src = _strip_c_comments(open(HEADER).read())
    src = re.sub(r"^\s*#.*$", " ", src, flags=re.M)  # preprocessor lines (#define ...)
    src = re.sub(r"\s+", " ", src)
    out = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z_0-9 ]*?)\s*(\*?)\s*\b(dips_\w+)\(([^)]*)\);", src):
        ret, star, name, args = m.group(1), m.group(2), m.group(3), m.group(4)
        ret = (ret + " " + star).strip()
        params = [] if args.strip() in ("", "void") else [_c_to_rust(a) for a in args.split(",")]
        out[name] = (_c_ret(ret), params)
    return out


def rust_structs():
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive[^\]]*\]\s*)?pub struct (\w+) \{(.*?)\}", src, flags=re.S):
        fields = re.findall(r"pub (\w+): ([^,]+),", m.group(2))
        out[m.group(1)] = [(f, t.strip()) for f, t in fields]
    return out


def _norm(t):
    return re.sub(r"\s+", " ", t.strip()) if t else None


def rust_functions():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    block = re.sub(r"//[^\n]*", " ", block)
    out = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        params = [p.split(":", 1)[1] for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = (_norm(m.group(3)), [_norm(p) for p in params])
    return out


def test_structs_match_header():
    h, r = header_structs(), rust_structs()
    for c_name, r_name in STRUCTS.items():
        assert r[r_name] == h[c_name], (c_name, r[r_name], h[c_name])


def test_functions_match_header():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 37
    assert set(r) == set(h), (set(h) - set(r), set(r) - set(h))
    for name, (ret, params) in h.items():
        assert r[name] == (ret, params), (name, r[name], (ret, params))


def _c_layout():
    """sizeof / offsetof of every field of the three structs, from gcc."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dips_hip.h"', "int main(void) {"]
    for c_name, fields in header_structs().items():
        lines.append(f'printf("{c_name} size %zu\\n", sizeof({c_name}));')
        for f, _ in fields:
            lines.append(f'printf("{c_name} {f} %zu\\n", offsetof({c_name}, {f}));')
    lines.append("return 0; }")
    return "\n".join(lines)


def test_rust_layout_asserts_match_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(_c_layout())
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-pedantic", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(exe)], check=True)
    c = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = line.split()
        c[(STRUCTS[s], f)] = int(v)
    rs = open(FFI).read()
    r = {}
    for name, v in re.findall(r"assert!\(size_of::<(\w+)>\(\) == (\d+)\);", rs):
        r[(name, "size")] = int(v)
    for name, f, v in re.findall(r"assert!\(offset_of!\((\w+), (\w+)\) == (\d+)\);", rs):
        r[(name, f)] = int(v)
    assert r == c


def test_header_layout_asserts_compile(tmp_path):
    """DIPS_LAYOUT_ASSERT holds in C99 and C++17 (a wrong size fails the build)."""
    src = tmp_path / "inc.c"
    src.write_text('#include "dips_hip.h"\nint main(void) { return 0; }\n')
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Werror", "-I", inc, "-c", str(src), "-o",
                    str(tmp_path / "a.o")], check=True)
    subprocess.run(["g++", "-std=c++17", "-Werror", "-x", "c++", "-I", inc, "-c", str(src), "-o",
                    str(tmp_path / "b.o")], check=True)
    bad = tmp_path / "bad.c"
    bad.write_text('#include "dips_hip.h"\nDIPS_LAYOUT_ASSERT(sizeof(dips_params) == 40, "x");\n')
    r = subprocess.run(["gcc", "-std=c99", "-I", inc, "-c", str(bad), "-o", str(tmp_path / "c.o")],
                       capture_output=True)
    assert r.returncode != 0


def test_filter_codes_match_reference_into_f64():
    """`Into<f64>` of DiPsFilter / ChromaFilter (dips/src/lib.rs:32-61): the
    crate's code() values are the header's constants and the reference's."""
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    consts = dict(re.findall(r"pub const (DIPS_\w+): u32 = (\w+);", open(FFI).read()))
    want = {"Unfiltered": 255, "Sigmoid": 0, "InverseSigmoid": 1, "None": 0, "Red": 1, "Green": 2, "Blue": 3}
    for variant, const in re.findall(r"(?:DiPsFilter|ChromaFilter)::(\w+) => ffi::(DIPS_\w+),", src):
        assert int(consts[const], 0) == want[variant], (variant, const)
    hdr = open(HEADER).read()
    for name, v in consts.items():
        m = re.search(r"#define %s (\w+?)u?\b" % name, hdr)
        assert m and int(m.group(1).rstrip("u"), 0) == int(v, 0), name


def test_crate_files_and_integration_doc():
    for p in ("Cargo.toml", "build.rs", "src/lib.rs", "src/ffi.rs", "examples/frame_callback.rs"):
        assert os.path.exists(os.path.join(CRATE, p)), p
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "rust/dips-hip" in doc
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    # the reference's operator surface, same names
    for sig in ("pub fn new(colorize: bool, spatial_window_size: i32, sensitivity: f32, filter_type: DiPsFilter,",
                "pub fn add_texture(&mut self, width: u32, height: u32, frame_data: &[u8])",
                "pub fn dispatch(&mut self) -> Option<Vec<u8>>",
                "pub fn frame_callback(width: u32, height: u32, frame_data: &[u8], compute: &mut ComputeState) -> Vec<u8>"):
        assert sig in lib, sig


def _fn_body(src, sig):
    """The body of the Rust fn whose signature starts with `sig` (brace matched)."""
    i = src.index(sig)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError("unbalanced braces after " + sig)


def test_failures_are_visible_at_the_rust_boundary():
    """a device error must not look like the warm-up.
    `try_dispatch` returns every failure; `dispatch` (the reference's
    signature, gpu/mod.rs:306-397) gives None only for the warm-up and panics
    on a negative status like the reference's wgpu path; `frame_callback`
    (lib.rs:233-246) panics instead of passing the input through."""
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    assert "pub fn try_dispatch(&mut self) -> Result<Option<Vec<u8>>, DipsError>" in lib
    assert "pub fn try_start_texture(&mut self) -> Result<Option<Vec<u8>>, DipsError>" in lib
    body = _fn_body(lib, "pub fn try_dispatch(")
    assert "check(r, self.h.as_ptr())?" in body  # negative status -> Err before the 1/0 match
    body = _fn_body(lib, "pub fn dispatch(&mut self)")
    assert "self.try_dispatch()" in body and "panic!" in body
    body = _fn_body(lib, "pub fn frame_callback(width: u32")
    assert "panic!" in body and "frame_data.to_vec()" not in body
    ffi = open(FFI).read()
    assert "pub const DIPS_ERR_INTERNAL: DipsStatus = -7;" in ffi
    assert "pub const DIPS_ABI_VERSION: c_int = 3;" in ffi
    assert "pub const DIPS_FLAG_CROSSCHECK: u32 = 0x8;" in ffi


def _rust_files():
    base = os.path.join(ROOT, "rust", "dips-hip")
    out = []
    for d, _, fs in os.walk(base):
        out += [os.path.join(d, f) for f in sorted(fs) if f.endswith(".rs")]
    return out


def test_rust_sources_lex_cleanly_and_balance():
    """No cargo / rustc in the image, so the crate is checked lexically:
    pygments' Rust lexer finds no error token in any .rs file, and every
    (), [] and {} outside strings, chars and comments closes in order."""
    from pygments.lexers import RustLexer
    from pygments.token import Comment, Error, String
    files = _rust_files()
    assert len(files) >= 3, files
    pairs = {")": "(", "]": "[", "}": "{"}
    for path in files:
        with open(path) as f:
            src = f.read()
        stack = []
        for ttype, value in RustLexer().get_tokens(src):
            assert ttype is not Error and ttype not in Error, (path, value)
            if ttype in String or ttype in Comment:
                continue
            for ch in value:
                if ch in "([{":
                    stack.append(ch)
                elif ch in ")]}":
                    assert stack and stack[-1] == pairs[ch], (path, ch)
                    stack.pop()
        assert not stack, (path, stack)


def test_rust_calls_only_declared_ffi():
    """Every ffi::dips_* the safe wrapper and the examples call is declared
    in ffi.rs (itself checked against the header above)."""
    ffi = _read(os.path.join(ROOT, "rust", "dips-hip", "src", "ffi.rs"))
    declared = set(re.findall(r"pub fn (dips_\w+)\(", ffi))
    for path in _rust_files():
        if path.endswith("ffi.rs"):
            continue
        for name in re.findall(r"ffi::(dips_\w+)\s*\(", _read(path)):
            assert name in declared, (path, name)


def _read(path):
    with open(path) as f:
        return f.read()


# Every method of the crate: the C entry point it calls, the status handling
# it implements (a token its body must contain) and the rows of
# tests/rust_contract.cpp that execute the same sequence
# (tests/test_rust_contract.py: CPU rows without a device, all rows on the GPU).
METHOD_TABLE = [
    # (signature prefix in lib.rs, C entry point, handling token, contract rows)
    ("fn check_abi(", "dips_abi_version", "ffi::DIPS_ERR_STATE", ["check_abi"]),
    ("fn create(", "dips_create", "check(unsafe { ffi::dips_create(p, device, &mut h) }, ptr::null())?",
     ["new", "diff_series_new"]),
    ("pub fn on_device(colorize", "dips_create", "create(&p, device)?", ["new"]),
    ("pub fn try_add_texture(", "dips_add_texture", "check(st, self.h.as_ptr())?", ["try_add_texture_error"]),
    ("pub fn add_texture(", "dips_add_texture", "let _ = self.try_add_texture", ["try_add_texture_error"]),
    ("pub fn try_dispatch(", "dips_dispatch", "check(r, self.h.as_ptr())?",
     ["try_dispatch_warmup", "try_dispatch_some", "try_dispatch_error"]),
    ("pub fn dispatch(&mut self)", "dips_dispatch", "panic!", ["dispatch_panics"]),
    ("pub fn frame_callback_into(", "dips_frame_callback", "check(r, self.h.as_ptr())?",
     ["frame_callback_into_size_change", "frame_callback_into_ok"]),
    ("pub fn frame_callback_batch(", "dips_frame_callback_batch", "check(st, self.h.as_ptr())?",
     ["frame_callback_batch"]),
    ("pub fn callback_phases(", "dips_callback_phases", "if st == ffi::DIPS_OK { Some(v) } else { None }",
     ["callback_phases", "callback_phases_after_call"]),
    ("pub fn try_start_texture(", "dips_start_texture", "check(r, self.h.as_ptr())?", ["try_start_texture"]),
    ("pub fn start_texture(", "dips_start_texture", "panic!", ["start_texture"]),
    ("pub fn resume(", "dips_compat_resume", "check(st, self.h.as_ptr())?", ["resume"]),
    ("pub fn frame_callback_batch_sharded(", "dips_frame_callback_batch_sharded", "check(st, self.h.as_ptr())?",
     ["frame_callback_batch_sharded"]),
    ("pub fn frame_callback(width: u32", "dips_frame_callback", "panic!", ["frame_callback_panics"]),
    ("pub fn run(&mut self, width: u32", "dips_diff_series", "check(st, self.h.as_ptr())?",
     ["diff_series_run", "diff_series_refusals"]),
    ("pub fn run_streamed(", "dips_diff_series_streamed", "check(st, self.h.as_ptr())?",
     ["diff_series_run_streamed"]),
    ("pub fn run_sharded(", "dips_diff_series_sharded", "check(st, self.h.as_ptr())?",
     ["diff_series_run_sharded", "diff_series_run_sharded_error"]),
    ("pub fn unique_id(", "dips_comm_unique_id", "check_comm(", ["comm_rccl"]),
    ("pub fn rccl(", "dips_comm_create", "check_comm(", ["comm_rccl", "comm_rccl_error"]),
    ("pub fn loopback(", "dips_comm_create_loopback", "check_comm(", ["comm_loopback"]),
    ("pub fn rccl_all(", "dips_comm_create_all", "check_comm(", ["comm_rccl_all"]),
    ("pub fn shard_range(", "dips_shard_range", "if st == ffi::DIPS_OK", ["shard_range"]),
    ("pub fn series_si(", "dips_series_si", "ffi::dips_series_si(e)", ["series_si"]),
    ("pub fn abi_version(", "dips_abi_version", "ffi::dips_abi_version()", ["series_si"]),
    ("pub fn new(num_textures", "dips_alt_create", "check_alt(", ["dips_compute_new"]),
    ("pub fn send_frame(", "dips_alt_send_frame", "check_alt(st, self.h.as_ptr())?", ["dips_compute_send_frame"]),
    ("pub fn run(&mut self, frames: &[u8], refresh_markers", "dips_alt_run", "check_alt(st, self.h.as_ptr())?",
     ["dips_compute_run"]),
    ("pub fn run_sharded(&mut self, comm: &mut Comm, frames", "dips_alt_run_sharded",
     "check_alt(st, self.h.as_ptr())?", ["dips_compute_run_sharded", "dips_compute_run_sharded_error"]),
]


def test_crate_method_table():
    """each crate method calls the C entry point the
    table names (directly or, for on_device / add_texture / dispatch /
    start_texture / frame_callback, through the method that does), carries
    the status handling named, and has rows in tests/rust_contract.cpp."""
    from test_rust_contract import contract_rows
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    rows = contract_rows()
    indirect = {"pub fn on_device(colorize": "create(", "pub fn add_texture(": "self.try_add_texture",
                "pub fn dispatch(&mut self)": "self.try_dispatch()", "pub fn start_texture(": "self.try_start_texture()",
                "pub fn frame_callback(width: u32": "compute.frame_callback_into("}
    for sig, entry, token, want_rows in METHOD_TABLE:
        body = _fn_body(lib, sig)
        via = indirect.get(sig)
        assert (f"ffi::{entry}(" in body) or (via and via in body), (sig, entry)
        assert token in body, (sig, token)
        for r in want_rows:
            assert r in rows, (sig, r)
    # every pub fn of the crate has a row (methods and free functions)
    pub = set(re.findall(r"pub fn (\w+)\(", lib))
    covered = {re.match(r"(?:pub )?fn (\w+)\(", sig).group(1) for sig, *_ in METHOD_TABLE}
    assert pub <= covered | {"code", "channels", "new"}, pub - covered
