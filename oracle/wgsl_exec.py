"""A WGSL-subset interpreter -- TEST INFRASTRUCTURE ONLY (oracle pinning).

The reference computes its visual operators in WGSL compute shaders run by
wgpu 24 / naga 24 (dips/src/gpu/shaders/*.wgsl,
dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl).  Neither Rust nor
a WebGPU implementation exists in this image, so the C and
numpy oracles are restatements of those shaders as read.  This module
executes the shader TEXT itself on the CPU, so that a restatement error (a
misread loop bound, an operator precedence, an abstract-literal conversion,
an index) shows up as a byte mismatch against the oracle instead of being
copied into both restatements.

What the WGSL specification leaves to the implementation is not guessed here
but passed in as explicit parameters (`Pins`), the same pins the oracle's
fixture manifest records:

* bounds policy for a runtime-indexed function-scope array
  (naga `Restrict`: clamp the index to the last element, the Vulkan / DX12
  backends; `ReadZeroSkipWrite`: read 0 / drop the write, Metal);
* rgba8unorm store rounding (round half to even, or half up) and NaN -> 0;
* rgba8unorm load = c / 255.0f in IEEE f32;
* exp / log: the oracle's deterministic f32 algorithms, or the correctly
  rounded f32 result (WGSL only bounds their error);
* order of a dispatch's invocations: all invocations run in lock step, so a
  load another invocation races with sees the texel as it was before the
  statement that stores it (the in-place spatial filter of
  dips_shader.wgsl:187 is such a race; this is the "reads see the slot as it
  was before the dispatch" pin).

Execution model: one dispatch is evaluated for all its invocations at once.
Every run-time value is a numpy array with a leading invocation axis (or a
uniform 0-d value); control flow runs under an active-lane mask (if / else,
for / while with break / continue, switch, return), f32 arithmetic is numpy
float32 (IEEE, round to nearest even, no FMA contraction -- also a pin), i32
/ u32 wrap.  The subset is what the reference's shaders use: module-scope
`var` bindings (storage textures, binding arrays of them, uniform u32),
`override` (with @id) and `const` declarations, functions with scalar,
vector, texture parameters, `var` / `let` / `const` statements, f32 / i32 /
u32 / bool scalars, vec2-4, fixed-size arrays of scalars, swizzles,
abstract-int / abstract-float literals with WGSL's conversion rules,
textureLoad / textureStore / textureDimensions, max / min / abs / clamp /
exp / log / select and the usual operators.  Anything else raises.

Only tests/ and tests/golden/ generator scripts use this module; nothing in
the product imports it.
"""
from __future__ import annotations

import dataclasses
import re
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

F32 = np.float32

# --------------------------------------------------------------------------
# implementation-defined behaviour, as explicit parameters
# --------------------------------------------------------------------------


@dataclasses.dataclass(frozen=True)
class Pins:
    bounds: str = "restrict"          # or "read_zero_skip_write"
    store_round: str = "half_even"    # or "half_up"
    exp_log: str = "oracle"           # or "nearest"

    def __post_init__(self):
        assert self.bounds in ("restrict", "read_zero_skip_write"), self.bounds
        assert self.store_round in ("half_even", "half_up"), self.store_round
        assert self.exp_log in ("oracle", "nearest"), self.exp_log


PINS = Pins()


class WgslError(Exception):
    pass


# --------------------------------------------------------------------------
# lexer
# --------------------------------------------------------------------------

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<comment>//[^\n]*|/\*.*?\*/)
  | (?P<num>0[xX][0-9a-fA-F]+[iu]?|(?:\d+\.\d*|\.\d+)(?:[eE][+-]?\d+)?[fh]?|\d+[eE][+-]?\d+[fh]?|\d+[iuf]?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>->|\+\+|--|&&|\|\||==|!=|<=|>=|\+=|-=|\*=|/=|%=|&=|\|=|\^=|[-+*/%<>=!&|^~(){}\[\];:,.@])
""", re.S | re.X)


def tokenize(src: str) -> List[tuple]:
    out, pos = [], 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise WgslError(f"unexpected character {src[pos]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment"):
            continue
        out.append((kind, m.group(kind)))
    out.append(("eof", ""))
    return out


# --------------------------------------------------------------------------
# parser (AST = tuples)
# --------------------------------------------------------------------------

_TYPE_GENERATORS = {"vec2", "vec3", "vec4", "array", "texture_storage_2d", "binding_array", "ptr", "atomic"}
_SCALARS = {"f32", "i32", "u32", "bool"}


class Parser:
    def __init__(self, src: str):
        self.t = tokenize(src)
        self.i = 0

    # token helpers
    def peek(self, k=0):
        return self.t[self.i + k]

    def at(self, text, k=0):
        return self.t[self.i + k][1] == text and self.t[self.i + k][0] in ("op", "id")

    def take(self, text=None):
        tok = self.t[self.i]
        if text is not None and tok[1] != text:
            raise WgslError(f"expected {text!r}, got {tok[1]!r} (token {self.i})")
        self.i += 1
        return tok

    def ident(self):
        tok = self.take()
        if tok[0] != "id":
            raise WgslError(f"expected identifier, got {tok[1]!r}")
        return tok[1]

    # module
    def module(self):
        decls = []
        while self.peek()[0] != "eof":
            attrs = self.attributes()
            if self.at("var"):
                self.take("var")
                space = None
                if self.at("<"):
                    self.take("<")
                    space = self.ident()
                    while not self.at(">"):
                        self.take()
                    self.take(">")
                name = self.ident()
                self.take(":")
                ty = self.type_()
                self.take(";")
                decls.append(("global_var", name, ty, space, attrs))
            elif self.at("override") or self.at("const"):
                kw = self.take()[1]
                name = self.ident()
                ty = None
                if self.at(":"):
                    self.take(":")
                    ty = self.type_()
                init = None
                if self.at("="):
                    self.take("=")
                    init = self.expr()
                self.take(";")
                decls.append((kw, name, ty, init, attrs))
            elif self.at("fn"):
                decls.append(self.function(attrs))
            elif self.at(";"):
                self.take(";")
            else:
                raise WgslError(f"unexpected {self.peek()[1]!r} at module scope")
        return decls

    def attributes(self):
        attrs = {}
        while self.at("@"):
            self.take("@")
            name = self.ident()
            args = []
            if self.at("("):
                self.take("(")
                while not self.at(")"):
                    args.append(self.expr())
                    if self.at(","):
                        self.take(",")
                self.take(")")
            attrs[name] = args
        return attrs

    def function(self, attrs):
        self.take("fn")
        name = self.ident()
        self.take("(")
        params = []
        while not self.at(")"):
            pattrs = self.attributes()
            pname = self.ident()
            self.take(":")
            params.append((pname, self.type_(), pattrs))
            if self.at(","):
                self.take(",")
        self.take(")")
        ret = None
        if self.at("->"):
            self.take("->")
            self.attributes()
            ret = self.type_()
        body = self.block()
        return ("fn", name, params, ret, body, attrs)

    def type_(self):
        name = self.ident()
        args = []
        if self.at("<"):
            self.take("<")
            while not self.at(">"):
                if self.peek()[0] == "id":
                    args.append(self.type_())
                else:
                    args.append(("lit_arg", self.primary()))
                if self.at(","):
                    self.take(",")
            self.take(">")
        return ("type", name, args)

    # statements
    def block(self):
        self.take("{")
        stmts = []
        while not self.at("}"):
            stmts.append(self.statement())
        self.take("}")
        return ("block", stmts)

    def statement(self):
        if self.at("{"):
            return self.block()
        if self.at(";"):
            self.take(";")
            return ("block", [])
        if self.at("var") or self.at("let") or self.at("const"):
            s = self.decl_stmt()
            self.take(";")
            return s
        if self.at("if"):
            return self.if_stmt()
        if self.at("for"):
            self.take("for")
            self.take("(")
            init = None if self.at(";") else self.simple_stmt()
            self.take(";")
            cond = None if self.at(";") else self.expr()
            self.take(";")
            upd = None if self.at(")") else self.simple_stmt()
            self.take(")")
            return ("for", init, cond, upd, self.block())
        if self.at("while"):
            self.take("while")
            cond = self.expr()
            return ("for", None, cond, None, self.block())
        if self.at("switch"):
            self.take("switch")
            sel = self.expr()
            self.take("{")
            clauses = []
            while not self.at("}"):
                sels = []
                if self.at("default"):
                    self.take("default")
                    sels.append(None)
                else:
                    self.take("case")
                    while True:
                        if self.at("default"):
                            self.take("default")
                            sels.append(None)
                        else:
                            sels.append(self.expr())
                        if self.at(","):
                            self.take(",")
                            if self.at(":") or self.at("{"):
                                break
                            continue
                        break
                if self.at(":"):
                    self.take(":")
                clauses.append((sels, self.block()))
            self.take("}")
            return ("switch", sel, clauses)
        if self.at("break"):
            self.take("break")
            self.take(";")
            return ("break",)
        if self.at("continue"):
            self.take("continue")
            self.take(";")
            return ("continue",)
        if self.at("return"):
            self.take("return")
            e = None if self.at(";") else self.expr()
            self.take(";")
            return ("return", e)
        s = self.simple_stmt()
        self.take(";")
        return s

    def decl_stmt(self):
        kw = self.take()[1]
        if kw == "var" and self.at("<"):
            while not self.at(">"):
                self.take()
            self.take(">")
        name = self.ident()
        ty = None
        if self.at(":"):
            self.take(":")
            ty = self.type_()
        init = None
        if self.at("="):
            self.take("=")
            init = self.expr()
        return ("decl", kw, name, ty, init)

    def simple_stmt(self):
        if self.at("var") or self.at("let") or self.at("const"):
            return self.decl_stmt()
        lhs = self.expr()
        if self.at("++") or self.at("--"):
            op = self.take()[1]
            return ("assign", lhs, "+" if op == "++" else "-", ("lit", "aint", 1))
        for op in ("=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^="):
            if self.at(op):
                self.take(op)
                return ("assign", lhs, None if op == "=" else op[0], self.expr())
        return ("expr", lhs)

    def if_stmt(self):
        self.take("if")
        cond = self.expr()
        then = self.block()
        other = None
        if self.at("else"):
            self.take("else")
            other = self.if_stmt() if self.at("if") else self.block()
        return ("if", cond, then, other)

    # expressions
    _BIN = [("||",), ("&&",), ("|",), ("^",), ("&",), ("==", "!="), ("<", ">", "<=", ">="), ("+", "-"),
            ("*", "/", "%")]

    def expr(self, level=0):
        if level == len(self._BIN):
            return self.unary()
        lhs = self.expr(level + 1)
        while self.peek()[0] == "op" and self.peek()[1] in self._BIN[level]:
            op = self.take()[1]
            rhs = self.expr(level + 1)
            lhs = ("bin", op, lhs, rhs)
        return lhs

    def unary(self):
        if self.peek()[0] == "op" and self.peek()[1] in ("-", "!", "~"):
            op = self.take()[1]
            return ("un", op, self.unary())
        return self.postfix(self.primary())

    def postfix(self, e):
        while True:
            if self.at("["):
                self.take("[")
                idx = self.expr()
                self.take("]")
                e = ("index", e, idx)
            elif self.at(".") and self.peek()[0] == "op":
                self.take(".")
                e = ("member", e, self.ident())
            else:
                return e

    def primary(self):
        kind, text = self.peek()
        if kind == "num":
            self.take()
            return parse_number(text)
        if self.at("("):
            self.take("(")
            e = self.expr()
            self.take(")")
            return e
        if kind == "id":
            if text in ("true", "false"):
                self.take()
                return ("lit", "bool", text == "true")
            if text in _TYPE_GENERATORS and self.at("<", 1):
                ty = self.type_()
                return ("call", ty, self.call_args())
            self.take()
            if self.at("("):
                return ("call", ("type", text, []) if text in _SCALARS or text in _TYPE_GENERATORS else text,
                        self.call_args())
            return ("ident", text)
        raise WgslError(f"unexpected {text!r} in expression")

    def call_args(self):
        self.take("(")
        args = []
        while not self.at(")"):
            args.append(self.expr())
            if self.at(","):
                self.take(",")
        self.take(")")
        return args


def parse_number(text: str):
    t = text.lower()
    if t.startswith("0x"):
        suf = t[-1] if t[-1] in "iu" else ""
        v = int(t[:-1] if suf else t, 16)
        return ("lit", {"i": "i32", "u": "u32", "": "aint"}[suf], v)
    if t[-1] in "iu":
        return ("lit", "i32" if t[-1] == "i" else "u32", int(t[:-1]))
    if t[-1] in "fh":
        return ("lit", "f32", float(t[:-1]))
    if any(c in t for c in ".e"):
        return ("lit", "afloat", float(t))
    return ("lit", "aint", int(t))


# --------------------------------------------------------------------------
# types and values
# --------------------------------------------------------------------------

_NP = {"f32": np.float32, "i32": np.int32, "u32": np.uint32, "bool": np.bool_}
_ABSTRACT = ("aint", "afloat")


class Texture:
    """An rgba8unorm 2D storage texture: uint8 [H, W, 4] (row = y)."""

    def __init__(self, data: np.ndarray):
        data = np.asarray(data)
        assert data.dtype == np.uint8 and data.ndim == 3 and data.shape[2] == 4, data.shape
        self.data = data

    @property
    def width(self):
        return self.data.shape[1]

    @property
    def height(self):
        return self.data.shape[0]


class V:
    """A value: WGSL type + numpy data.  Scalars: [P] or 0-d; vectors
    [P, n] or [n]; arrays [P, N] or [N]; abstract literals: python numbers;
    textures / binding arrays: Texture / list."""
    __slots__ = ("ty", "d")

    def __init__(self, ty, d):
        self.ty = ty
        self.d = d

    def __repr__(self):
        return f"V({self.ty}, {self.d!r})"


def scalar_of(ty):
    if isinstance(ty, str):
        return ty
    if ty[0] == "vec":
        return ty[2]
    raise WgslError(f"not a numeric type: {ty}")


def _as(d, s):
    """numpy data -> scalar type s (value conversion of an abstract / same kind)."""
    if s == "f32":
        return np.asarray(d, dtype=np.float32) if not isinstance(d, (int, float)) else F32(d)
    if s == "i32":
        return np.asarray(d).astype(np.int32) if not isinstance(d, int) else np.int32(np.int64(d).astype(np.int32))
    if s == "u32":
        return np.asarray(d).astype(np.uint32) if not isinstance(d, int) else np.uint32(d & 0xFFFFFFFF)
    if s == "bool":
        return np.asarray(d, dtype=np.bool_)
    raise WgslError(s)


def concretize(v: V, target: Optional[str] = None) -> V:
    """Abstract -> concrete (default i32 / f32, or the given scalar type)."""
    if isinstance(v.ty, str) and v.ty in _ABSTRACT:
        s = target or ("i32" if v.ty == "aint" else "f32")
        if v.ty == "afloat" and s in ("i32", "u32"):
            raise WgslError("abstract float cannot convert to an integer type")
        return V(s, _as(v.d, s))
    return v


def convert_to(v: V, ty) -> V:
    """Implicit conversion of v to the declared type ty (abstract only)."""
    if ty is None:
        return concretize(v)
    if isinstance(ty, str):
        if isinstance(v.ty, str) and v.ty in _ABSTRACT:
            return concretize(v, ty)
        if v.ty != ty:
            raise WgslError(f"type mismatch: {v.ty} vs {ty}")
        return v
    if ty[0] == "vec" and isinstance(v.ty, tuple) and v.ty[0] == "vec":
        if v.ty != ty:
            raise WgslError(f"type mismatch: {v.ty} vs {ty}")
        return v
    return v


# --------------------------------------------------------------------------
# arithmetic
# --------------------------------------------------------------------------

def _int_div(a, b, s):
    a64, b64 = np.asarray(a).astype(np.int64), np.asarray(b).astype(np.int64)
    zero = b64 == 0
    bb = np.where(zero, 1, b64)
    q = np.abs(a64) // np.abs(bb) * np.sign(a64) * np.sign(bb)
    if s == "i32":
        q = np.where(zero | ((a64 == -2 ** 31) & (b64 == -1)), a64, q)
    else:
        q = np.where(zero, a64, q)
    return q


def _int_rem(a, b, s):
    a64, b64 = np.asarray(a).astype(np.int64), np.asarray(b).astype(np.int64)
    zero = b64 == 0
    bb = np.where(zero, 1, b64)
    q = np.abs(a64) // np.abs(bb) * np.sign(a64) * np.sign(bb)
    r = a64 - bb * q
    return np.where(zero | ((s == "i32") & (a64 == -2 ** 31) & (b64 == -1)), 0, r)


def _abstract_binop(op, a, b, ta, tb):
    isf = "afloat" in (ta, tb)
    if op in ("==", "!=", "<", ">", "<=", ">="):
        r = {"==": a == b, "!=": a != b, "<": a < b, ">": a > b, "<=": a <= b, ">=": a >= b}[op]
        return V("bool", np.bool_(r))
    if op in ("&&", "||"):
        raise WgslError("logical op on numbers")
    ty = "afloat" if isf else "aint"
    if op == "+":
        r = a + b
    elif op == "-":
        r = a - b
    elif op == "*":
        r = a * b
    elif op == "/":  # abstract ints: truncating (a zero divisor is a shader-creation error)
        r = a / b if isf else abs(a) // abs(b) * (1 if (a >= 0) == (b > 0) else -1)
    elif op == "%":
        r = a - b * int(a / b) if isf else a - b * (abs(a) // abs(b) * (1 if (a >= 0) == (b > 0) else -1))
    elif op in ("&", "|", "^") and not isf:
        r = {"&": a & b, "|": a | b, "^": a ^ b}[op]
    else:
        raise WgslError(f"abstract {op}")
    return V(ty, float(r) if isf else int(r))


def binop(op: str, a: V, b: V) -> V:
    if isinstance(a.ty, str) and isinstance(b.ty, str) and a.ty in _ABSTRACT and b.ty in _ABSTRACT:
        return _abstract_binop(op, a.d, b.d, a.ty, b.ty)
    if op in ("&&", "||"):
        if a.ty != "bool" or b.ty != "bool":
            raise WgslError(f"{op} on {a.ty}, {b.ty}")
        return V("bool", np.logical_and(a.d, b.d) if op == "&&" else np.logical_or(a.d, b.d))
    # concretize the abstract side to the concrete side's scalar type
    sa = None if (isinstance(a.ty, str) and a.ty in _ABSTRACT) else scalar_of(a.ty)
    sb = None if (isinstance(b.ty, str) and b.ty in _ABSTRACT) else scalar_of(b.ty)
    s = sa or sb
    if sa is None:
        a = concretize(a, s)
    if sb is None:
        b = concretize(b, s)
    if scalar_of(a.ty) != scalar_of(b.ty):
        raise WgslError(f"{op}: {a.ty} vs {b.ty}")
    ad, bd = a.d, b.d
    # vector-scalar broadcasting
    va = isinstance(a.ty, tuple)
    vb = isinstance(b.ty, tuple)
    rty = a.ty if va else b.ty
    if va and not vb:
        bd = np.asarray(bd)[..., None]
    if vb and not va:
        ad = np.asarray(ad)[..., None]
    if op in ("==", "!=", "<", ">", "<=", ">="):
        r = {"==": np.equal, "!=": np.not_equal, "<": np.less, ">": np.greater, "<=": np.less_equal,
             ">=": np.greater_equal}[op](ad, bd)
        return V(("vec", rty[1], "bool") if isinstance(rty, tuple) else "bool", r)
    dt = _NP[s]
    if s == "f32":
        if op == "+":
            r = np.add(ad, bd, dtype=np.float32)
        elif op == "-":
            r = np.subtract(ad, bd, dtype=np.float32)
        elif op == "*":
            r = np.multiply(ad, bd, dtype=np.float32)
        elif op == "/":
            r = np.divide(ad, bd, dtype=np.float32)
        elif op == "%":  # e1 - e2 * trunc(e1 / e2), each step in f32
            r = np.subtract(ad, np.multiply(bd, np.trunc(np.divide(ad, bd, dtype=np.float32)), dtype=np.float32),
                            dtype=np.float32)
        else:
            raise WgslError(f"f32 {op}")
        return V(rty, r)
    if s == "bool":
        if op in ("&", "|", "^"):
            return V(rty, {"&": np.logical_and, "|": np.logical_or, "^": np.logical_xor}[op](ad, bd))
        raise WgslError(f"bool {op}")
    a64, b64 = np.asarray(ad).astype(np.int64), np.asarray(bd).astype(np.int64)
    if op == "+":
        r = a64 + b64
    elif op == "-":
        r = a64 - b64
    elif op == "*":
        r = a64 * b64
    elif op == "/":
        r = _int_div(a64, b64, s)
    elif op == "%":
        r = _int_rem(a64, b64, s)
    elif op == "&":
        r = a64 & b64
    elif op == "|":
        r = a64 | b64
    elif op == "^":
        r = a64 ^ b64
    else:
        raise WgslError(f"int {op}")
    return V(rty, np.asarray(r).astype(dt))  # two's-complement wrap


def unop(op: str, a: V) -> V:
    if isinstance(a.ty, str) and a.ty in _ABSTRACT:
        if op == "-":
            return V(a.ty, -a.d)
        if op == "~" and a.ty == "aint":
            return V("aint", ~a.d)
        raise WgslError(f"abstract unary {op}")
    s = scalar_of(a.ty)
    if op == "!":
        if s != "bool":
            raise WgslError("! on non-bool")
        return V(a.ty, np.logical_not(a.d))
    if op == "-":
        if s == "f32":
            return V(a.ty, np.negative(a.d, dtype=np.float32))
        return V(a.ty, (-np.asarray(a.d).astype(np.int64)).astype(_NP[s]))
    if op == "~":
        return V(a.ty, np.invert(a.d))
    raise WgslError(op)


# --------------------------------------------------------------------------
# interpreter
# --------------------------------------------------------------------------

class _Var:
    __slots__ = ("v", "mutable")

    def __init__(self, v, mutable):
        self.v = v
        self.mutable = mutable


class _Fn:
    def __init__(self, done, ret_ty):
        self.done = done          # lanes that have returned
        self.ret_ty = ret_ty
        self.ret = None


class _Loop:
    def __init__(self, P, is_switch=False):
        self.broken = np.zeros(P, dtype=bool)
        self.cont = np.zeros(P, dtype=bool)
        self.is_switch = is_switch


_SWIZ = {c: i for i, c in enumerate("xyzw")}
_SWIZ.update({c: i for i, c in enumerate("rgba")})


def _where(m, new, old):
    """Masked select with the mask over the leading (lane) axis."""
    new, old = np.asarray(new), np.asarray(old)
    nd = max(new.ndim, old.ndim)
    mm = m.reshape(m.shape + (1,) * (nd - 1)) if nd >= 1 else m
    return np.where(mm, new, old)


class Module:
    """A parsed WGSL module.  `pipeline(entry, constants)` resolves the
    overrides (pipeline constants keyed by @id number or by name, f64 values
    converted to the override's type as WebGPU does; keys the module does not
    declare are ignored -- the reference passes dips_shader's five constants
    to the pre-compute module too, gpu/mod.rs:105-126)."""

    def __init__(self, src: str):
        self.decls = Parser(src).module()
        self.fns = {d[1]: d for d in self.decls if d[0] == "fn"}

    def pipeline(self, entry: str, constants: Optional[Dict[str, float]] = None, pins: Pins = PINS):
        return Pipeline(self, entry, constants or {}, pins)


class Pipeline:
    def __init__(self, module: Module, entry: str, constants: Dict[str, float], pins: Pins):
        self.m = module
        self.pins = pins
        if entry not in module.fns:
            raise WgslError(f"no entry point {entry}")
        self.entry = module.fns[entry]
        self.globals: Dict[str, _Var] = {}
        self.bind_decls = {}
        self.P = 1
        self._ovr_values = {}
        for d in module.decls:
            if d[0] == "override":
                _, name, ty, init, attrs = d
                key = None
                if "id" in attrs:
                    key = str(self._const_int(attrs["id"][0]))
                val = None
                for k in (key, name):
                    if k is not None and k in constants:
                        val = constants[k]
                        break
                if val is not None:
                    rty = self.resolve_type(ty) if ty is not None else None
                    if rty is None:
                        raise WgslError(f"override {name} without a type given a constant")
                    v = self._from_f64(val, rty)
                else:
                    if init is None:
                        raise WgslError(f"override {name} has no value")
                    v = self.eval_const(init)
                    v = convert_to(v, self.resolve_type(ty) if ty is not None else None)
                self.globals[name] = _Var(v, False)
            elif d[0] == "const":
                _, name, ty, init, attrs = d
                v = self.eval_const(init)
                if ty is not None:
                    v = convert_to(v, self.resolve_type(ty))
                self.globals[name] = _Var(v, False)
            elif d[0] == "global_var":
                _, name, ty, space, attrs = d
                self.bind_decls[name] = (self.resolve_type(ty), space)

    # -- helpers for module-scope evaluation
    def _const_int(self, e):
        v = self.eval_const(e)
        return int(np.asarray(v.d))

    @staticmethod
    def _from_f64(x: float, ty):
        if ty == "bool":
            return V("bool", np.bool_(x != 0.0))
        if ty == "f32":
            return V("f32", F32(x))
        if ty in ("i32", "u32"):
            if float(x) != int(x):
                raise WgslError(f"pipeline constant {x} is not an integer")
            return V(ty, _as(int(x), ty))
        raise WgslError(f"override type {ty}")

    def eval_const(self, e):
        saved = getattr(self, "_scopes", None)
        self._scopes = [{}]
        self.P = 1
        try:
            return self.eval(e, np.ones(1, dtype=bool))
        finally:
            self._scopes = saved

    def resolve_type(self, t):
        if t is None:
            return None
        _, name, args = t
        if name in _SCALARS:
            return name
        if name in ("vec2", "vec3", "vec4"):
            return ("vec", int(name[3]), self.resolve_type(args[0]))
        if name == "array":
            elem = self.resolve_type(args[0])
            a = args[1]
            if a[0] == "lit_arg":
                n = int(a[1][2])
            else:
                n = int(np.asarray(self.globals[a[1]].v.d))
            return ("array", elem, n)
        if name == "texture_storage_2d":
            return ("tex", args[0][1], args[1][1])
        if name == "binding_array":
            return ("barray", self.resolve_type(args[0]))
        raise WgslError(f"type {name}")

    # -- dispatch
    def dispatch(self, bindings: Dict[str, Any], workgroups: Sequence[int]):
        """Run the entry point over workgroups (x, y, z) with the given
        bindings (Texture, list of Texture, or an int for a uniform u32)."""
        attrs = self.entry[5]
        ws = [self._const_int(a) for a in attrs.get("workgroup_size", [])]
        ws = (ws + [1, 1, 1])[:3]
        gx, gy, gz = (list(workgroups) + [1, 1, 1])[:3]
        nx, ny, nz = gx * ws[0], gy * ws[1], gz * ws[2]
        P = nx * ny * nz
        lane = np.arange(P, dtype=np.int64)
        gid = np.stack([lane % nx, (lane // nx) % ny, lane // (nx * ny)], axis=-1).astype(np.uint32)
        for name, (ty, space) in self.bind_decls.items():
            if name not in bindings:
                continue
            b = bindings[name]
            if ty[0] == "tex":
                v = V(ty, b)
            elif ty[0] == "barray":
                v = V(ty, list(b))
            else:
                v = V(ty, _as(int(b), ty) if ty in ("u32", "i32") else _as(b, ty))
            self.globals[name] = _Var(v, False)
        args = []
        for pname, pty, pattrs in self.entry[2]:
            bi = pattrs.get("builtin")
            if not bi or bi[0][1] != "global_invocation_id":
                raise WgslError(f"entry parameter {pname}: only global_invocation_id is supported")
            args.append(V(("vec", 3, "u32"), gid))
        with np.errstate(all="ignore"):
            self.P = P
            self._scopes = []
            self.call_fn(self.entry, args, np.ones(P, dtype=bool))

    def call(self, fn_name: str, args: Sequence[V]):
        """Evaluate a module function for P lanes of the given arguments."""
        P = 1
        for a in args:
            d = np.asarray(a.d) if not isinstance(a.d, (Texture, list)) else None
            if d is not None and d.ndim >= 1:
                P = max(P, d.shape[0])
        with np.errstate(all="ignore"):
            self.P = P
            self._scopes = []
            return self.call_fn(self.m.fns[fn_name], list(args), np.ones(P, dtype=bool))

    # -- scopes
    def lookup(self, name):
        for s in reversed(self._scopes):
            if name in s:
                return s[name]
        if name in self.globals:
            return self.globals[name]
        raise WgslError(f"unknown identifier {name}")

    # -- functions
    def call_fn(self, fn, args, mask):
        _, name, params, ret, body, attrs = fn
        saved_scopes, saved_ctx = self._scopes, getattr(self, "_ctx", None)
        scope = {}
        for (pname, pty, _), a in zip(params, args):
            rty = self.resolve_type(pty)
            if isinstance(rty, tuple) and rty[0] in ("tex", "barray"):
                scope[pname] = _Var(a, False)
            else:
                scope[pname] = _Var(convert_to(a, rty), False)
        self._scopes = [scope]
        fctx = _Fn(np.zeros(self.P, dtype=bool), self.resolve_type(ret))
        self._ctx = (fctx, [])
        try:
            self.exec_block(body, mask, new_scope=False)
        finally:
            self._scopes, self._ctx = saved_scopes, saved_ctx
        if fctx.ret_ty is not None:
            if fctx.ret is None:
                raise WgslError(f"{name}: no lane returned a value")
            return fctx.ret
        return None

    def alive(self, mask):
        fctx, loops = self._ctx
        m = mask & ~fctx.done
        if loops:
            lp = loops[-1]
            m = m & ~lp.broken & ~lp.cont
        return m

    def exec_block(self, blk, mask, new_scope=True):
        if new_scope:
            self._scopes.append({})
        try:
            for s in blk[1]:
                m = self.alive(mask)
                if not m.any():
                    break
                self.exec_stmt(s, m)
        finally:
            if new_scope:
                self._scopes.pop()

    def exec_stmt(self, s, m):
        k = s[0]
        if k == "block":
            self.exec_block(s, m)
        elif k == "decl":
            _, kw, name, ty, init = s
            rty = self.resolve_type(ty)
            if init is None:
                v = self.zero(rty)
            else:
                v = self.eval(init, m)
                if kw == "const":
                    v = convert_to(v, rty) if rty is not None else v
                else:
                    v = convert_to(v, rty)
                    if isinstance(v.ty, tuple) and v.ty[0] == "array":
                        v = V(v.ty, np.array(v.d, copy=True))
            self._scopes[-1][name] = _Var(v, kw == "var")
        elif k == "assign":
            _, lhs, op, rhs = s
            val = self.eval(rhs, m)
            if op is not None:
                val = binop(op, self.eval(lhs, m), val)
            self.store(lhs, val, m)
        elif k == "expr":
            self.eval(s[1], m)
        elif k == "if":
            _, cond, then, other = s
            c = self.eval(cond, m)
            if c.ty != "bool":
                raise WgslError("if condition is not bool")
            c = np.broadcast_to(np.asarray(c.d), m.shape)
            mt, mf = m & c, m & ~c
            if mt.any():
                self.exec_block(then, mt)
            if other is not None and mf.any():
                if other[0] == "if":
                    self.exec_stmt(other, self.alive(mf))
                else:
                    self.exec_block(other, self.alive(mf))
        elif k == "for":
            self.exec_for(s, m)
        elif k == "switch":
            _, sel, clauses = s
            sv = self.eval(sel, m)
            sv = concretize(sv)
            fctx, loops = self._ctx
            lp = _Loop(self.P, is_switch=True)
            taken = np.zeros(self.P, dtype=bool)
            default = None
            for sels, body in clauses:
                cm = np.zeros(self.P, dtype=bool)
                for e in sels:
                    if e is None:
                        default = body
                        continue
                    cm |= np.broadcast_to(np.asarray(binop("==", sv, self.eval(e, m)).d), m.shape)
                cm &= m & ~taken
                taken |= cm
                if cm.any():
                    loops.append(lp)
                    try:
                        self.exec_block(body, cm)
                    finally:
                        loops.pop()
            if default is not None:
                dm = m & ~taken
                if dm.any():
                    loops.append(lp)
                    try:
                        self.exec_block(default, dm)
                    finally:
                        loops.pop()
        elif k == "break":
            self._ctx[1][-1].broken |= m
        elif k == "continue":
            loops = self._ctx[1]
            for lp in reversed(loops):
                if not lp.is_switch:
                    lp.cont |= m
                    # a continue inside a switch leaves the switch as well
                    for inner in loops[loops.index(lp) + 1:]:
                        inner.broken |= m
                    break
        elif k == "return":
            fctx = self._ctx[0]
            if s[1] is not None:
                v = convert_to(self.eval(s[1], m), fctx.ret_ty)
                d = np.asarray(v.d)
                if fctx.ret is None:
                    shape = (self.P, v.ty[1]) if isinstance(v.ty, tuple) else (self.P,)
                    fctx.ret = V(v.ty, np.zeros(shape, dtype=_NP[scalar_of(v.ty)]))
                fctx.ret = V(fctx.ret.ty, _where(m, np.broadcast_to(d, fctx.ret.d.shape), fctx.ret.d))
            fctx.done = fctx.done | m
        else:
            raise WgslError(f"statement {k}")

    def exec_for(self, s, mask):
        _, init, cond, upd, body = s
        self._scopes.append({})
        try:
            if init is not None:
                self.exec_stmt(init, mask)
            fctx, loops = self._ctx
            lp = _Loop(self.P)
            for _ in range(1 << 20):
                m = mask & ~fctx.done & ~lp.broken
                if cond is not None and m.any():
                    c = np.broadcast_to(np.asarray(self.eval(cond, m).d), m.shape)
                    lp.broken |= m & ~c
                    m = m & c
                if not m.any():
                    return
                lp.cont[:] = False
                loops.append(lp)
                try:
                    self.exec_block(body, m)
                finally:
                    loops.pop()
                if upd is not None:
                    mu = mask & ~fctx.done & ~lp.broken
                    if mu.any():
                        self.exec_stmt(upd, mu)
            raise WgslError("loop did not terminate")
        finally:
            self._scopes.pop()

    def zero(self, ty):
        if isinstance(ty, str):
            return V(ty, np.zeros(self.P, dtype=_NP[ty]))
        if ty[0] == "vec":
            return V(ty, np.zeros((self.P, ty[1]), dtype=_NP[ty[2]]))
        if ty[0] == "array":
            if not isinstance(ty[1], str):
                raise WgslError("arrays of non-scalars are not supported")
            return V(ty, np.zeros((self.P, ty[2]), dtype=_NP[ty[1]]))
        raise WgslError(f"zero of {ty}")

    # -- stores
    def store(self, lhs, val, m):
        if lhs[0] == "ident":
            var = self.lookup(lhs[1])
            if not var.mutable:
                raise WgslError(f"assignment to immutable {lhs[1]}")
            old = var.v
            val = convert_to(val, old.ty)
            od = np.asarray(old.d)
            if od.ndim == 0 or od.shape[0] != self.P:
                od = np.broadcast_to(od, (self.P,) + od.shape).copy()
            nd = np.broadcast_to(np.asarray(val.d), od.shape)
            var.v = V(old.ty, _where(m, nd, od))
        elif lhs[0] == "index":
            base = lhs[1]
            if base[0] != "ident":
                raise WgslError("only arrays held by a variable can be indexed in a store")
            var = self.lookup(base[1])
            if not var.mutable:
                raise WgslError(f"assignment to immutable {base[1]}")
            arr = var.v
            if not (isinstance(arr.ty, tuple) and arr.ty[0] == "array"):
                raise WgslError("indexed store into a non-array")
            n = arr.ty[2]
            val = convert_to(val, arr.ty[1])
            idx = self._index(self.eval(lhs[2], m), n, m)
            data = arr.d
            if data.ndim == 1:
                data = np.broadcast_to(data, (self.P, n)).copy()
            rows = np.nonzero(m)[0]
            ii = np.broadcast_to(idx.ix, m.shape)[rows]
            ok = np.broadcast_to(idx.ok, m.shape)[rows]
            vals = np.broadcast_to(np.asarray(val.d), m.shape)[rows]
            data[rows[ok], ii[ok]] = vals[ok]  # read_zero_skip_write drops the rest
            var.v = V(arr.ty, data)
        else:
            raise WgslError(f"store to {lhs[0]}")

    class _Idx:
        __slots__ = ("ix", "ok")

        def __init__(self, ix, ok):
            self.ix, self.ok = ix, ok

    def _index(self, iv, n, m):
        """Bounds policy for a runtime index into an n-element array."""
        iv = concretize(iv)
        raw = np.asarray(iv.d).astype(np.int64)
        if scalar_of(iv.ty) == "i32":
            raw = raw & 0xFFFFFFFF  # naga compares the index as u32
        inb = raw < n
        if self.pins.bounds == "restrict":
            return self._Idx(np.minimum(raw, n - 1), np.ones_like(inb))
        return self._Idx(np.where(inb, raw, 0), inb)

    # -- expressions
    def eval(self, e, m):
        k = e[0]
        if k == "lit":
            _, ty, val = e
            if ty in _ABSTRACT:
                return V(ty, val)
            if ty == "bool":
                return V("bool", np.bool_(val))
            return V(ty, _as(val, ty))
        if k == "ident":
            return self.lookup(e[1]).v
        if k == "bin":
            return binop(e[1], self.eval(e[2], m), self.eval(e[3], m))
        if k == "un":
            return unop(e[1], self.eval(e[2], m))
        if k == "member":
            b = self.eval(e[1], m)
            if not (isinstance(b.ty, tuple) and b.ty[0] == "vec"):
                raise WgslError(f"member {e[2]} of {b.ty}")
            idx = [_SWIZ[c] for c in e[2]]
            d = np.asarray(b.d)
            if len(idx) == 1:
                return V(b.ty[2], d[..., idx[0]])
            return V(("vec", len(idx), b.ty[2]), d[..., idx])
        if k == "index":
            b = self.eval(e[1], m)
            iv = self.eval(e[2], m)
            if isinstance(b.ty, tuple) and b.ty[0] == "barray":
                vals = np.broadcast_to(np.asarray(concretize(iv).d), m.shape)[m]
                if vals.size == 0:
                    return V(b.ty[1], b.d[0])
                if not np.all(vals == vals[0]):
                    raise WgslError("non-uniform binding_array index")
                j = int(vals[0])
                if not 0 <= j < len(b.d):
                    raise WgslError("binding_array index out of range")
                return V(b.ty[1], b.d[j])
            if isinstance(b.ty, tuple) and b.ty[0] == "array":
                n = b.ty[2]
                idx = self._index(iv, n, m)
                d = np.asarray(b.d)
                if d.ndim == 1:
                    r = d[np.asarray(idx.ix)]
                else:
                    ix = np.broadcast_to(idx.ix, (d.shape[0],))
                    r = d[np.arange(d.shape[0]), ix]
                r = np.where(idx.ok, r, 0).astype(d.dtype)
                return V(b.ty[1], r)
            if isinstance(b.ty, tuple) and b.ty[0] == "vec":
                j = np.asarray(concretize(iv).d).astype(np.int64)
                d = np.asarray(b.d)
                j = np.minimum(j, b.ty[1] - 1)
                if d.ndim == 1:
                    return V(b.ty[2], d[j])
                return V(b.ty[2], np.take_along_axis(d, np.broadcast_to(j, d.shape[:1])[:, None], 1)[:, 0])
            raise WgslError(f"index into {b.ty}")
        if k == "call":
            return self.eval_call(e, m)
        raise WgslError(f"expression {k}")

    def eval_call(self, e, m):
        _, callee, argx = e
        if isinstance(callee, tuple):  # type constructor / conversion
            ty = self.resolve_type(callee)
            args = [self.eval(a, m) for a in argx]
            return self.construct(ty, args)
        name = callee
        if name in self.m.fns:
            args = [self.eval(a, m) for a in argx]
            return self.call_fn(self.m.fns[name], args, m)
        args = [self.eval(a, m) for a in argx]
        return self.builtin(name, args, m)

    def construct(self, ty, args):
        if isinstance(ty, str):  # scalar conversion
            if len(args) != 1:
                raise WgslError(f"{ty}() takes one argument")
            a = args[0]
            if isinstance(a.ty, str) and a.ty in _ABSTRACT:
                return concretize(a, ty) if not (a.ty == "afloat" and ty in ("i32", "u32")) else \
                    V(ty, _f2i(np.asarray(F32(a.d)), ty))
            s = scalar_of(a.ty)
            d = np.asarray(a.d)
            if ty == s:
                return a
            if ty == "f32":
                return V("f32", d.astype(np.float32))
            if ty in ("i32", "u32"):
                if s == "f32":
                    return V(ty, _f2i(d, ty))
                if s == "bool":
                    return V(ty, d.astype(_NP[ty]))
                return V(ty, d.astype(np.int64).astype(_NP[ty]))  # bit reinterpretation (wrap)
            if ty == "bool":
                return V("bool", d != 0)
            raise WgslError(f"conversion to {ty}")
        if ty[0] == "vec":
            n, s = ty[1], ty[2]
            comps = []
            for a in args:
                a = concretize(a, s) if isinstance(a.ty, str) and a.ty in _ABSTRACT else a
                d = np.asarray(a.d)
                if isinstance(a.ty, tuple):
                    if a.ty[2] != s:
                        d = _convert_data(d, a.ty[2], s)
                    for i in range(a.ty[1]):
                        comps.append(d[..., i])
                else:
                    if a.ty != s:
                        d = _convert_data(d, a.ty, s)
                    comps.append(d)
            if len(comps) == 1:
                comps = comps * n
            if len(comps) != n:
                raise WgslError(f"vec{n} constructor with {len(comps)} components")
            shape = np.broadcast_shapes(*[np.shape(c) for c in comps])
            return V(ty, np.stack([np.broadcast_to(c, shape) for c in comps], axis=-1).astype(_NP[s]))
        raise WgslError(f"constructor {ty}")

    def builtin(self, name, args, m):
        pins = self.pins
        if name in ("max", "min"):
            a, b = args
            v = binop("+", a, b)  # unify the types
            a = concretize(a, scalar_of(v.ty)) if isinstance(a.ty, str) and a.ty in _ABSTRACT else a
            b = concretize(b, scalar_of(v.ty)) if isinstance(b.ty, str) and b.ty in _ABSTRACT else b
            if isinstance(v.ty, str) and v.ty in _ABSTRACT:
                return V(v.ty, max(a.d, b.d) if name == "max" else min(a.d, b.d))
            f = {"max": np.fmax, "min": np.fmin} if scalar_of(v.ty) == "f32" else {"max": np.maximum,
                                                                                     "min": np.minimum}
            return V(v.ty, f[name](a.d, b.d).astype(_NP[scalar_of(v.ty)]))
        if name == "abs":
            (a,) = args
            if isinstance(a.ty, str) and a.ty in _ABSTRACT:
                return V(a.ty, abs(a.d))
            s = scalar_of(a.ty)
            if s == "f32":
                return V(a.ty, np.abs(a.d).astype(np.float32))
            return V(a.ty, np.abs(np.asarray(a.d).astype(np.int64)).astype(_NP[s]))
        if name == "clamp":
            x, lo, hi = args
            return self.builtin("min", [self.builtin("max", [x, lo], m), hi], m)
        if name == "select":
            f, t, c = args
            v = binop("+", f, t)
            f, t = concretize(f, scalar_of(v.ty)), concretize(t, scalar_of(v.ty))
            return V(v.ty, np.where(c.d, t.d, f.d))
        if name in ("exp", "log"):
            (a,) = args
            a = concretize(a, "f32")
            x = np.asarray(a.d, dtype=np.float32)
            if pins.exp_log == "oracle":
                from oracle import np_restatement as nr
                r = nr.expf(x) if name == "exp" else nr.logf(x)
            else:
                x64 = x.astype(np.float64)
                r = (np.exp(x64) if name == "exp" else np.log(x64)).astype(np.float32)
            return V(a.ty, np.asarray(r, dtype=np.float32))
        if name == "textureDimensions":
            (t,) = args
            tex = t.d
            return V(("vec", 2, "u32"), np.array([tex.width, tex.height], dtype=np.uint32))
        if name == "textureLoad":
            t, c = args[0], args[1]
            tex = t.d
            xy = np.asarray(concretize(c).d).astype(np.int64)
            x = np.broadcast_to(xy[..., 0], m.shape)
            y = np.broadcast_to(xy[..., 1], m.shape)
            bad = m & ((x < 0) | (x >= tex.width) | (y < 0) | (y >= tex.height))
            if bad.any():
                raise WgslError("textureLoad out of bounds")
            px = tex.data[np.clip(y, 0, tex.height - 1), np.clip(x, 0, tex.width - 1)]
            return V(("vec", 4, "f32"), px.astype(np.float32) / np.float32(255.0))
        if name == "textureStore":
            t, c, val = args
            tex = t.d
            xy = np.asarray(concretize(c).d).astype(np.int64)
            x = np.broadcast_to(xy[..., 0], m.shape)[m]
            y = np.broadcast_to(xy[..., 1], m.shape)[m]
            if ((x < 0) | (x >= tex.width) | (y < 0) | (y >= tex.height)).any():
                raise WgslError("textureStore out of bounds")
            v = np.broadcast_to(np.asarray(val.d, dtype=np.float32), m.shape + (4,))[m]
            tex.data[y, x] = unorm8_store(v, pins)
            return None
        raise WgslError(f"unknown function {name}")


def _f2i(d, ty):
    """f32 -> i32 / u32: truncate toward zero, saturate (NaN -> 0)."""
    d = np.asarray(d, dtype=np.float64)
    lo, hi = (-2.0 ** 31, 2.0 ** 31 - 128) if ty == "i32" else (0.0, 2.0 ** 32 - 256)
    r = np.trunc(np.clip(np.nan_to_num(d, nan=0.0), lo, hi))
    return r.astype(np.int64).astype(_NP[ty])


def _convert_data(d, s_from, s_to):
    if s_to == "f32":
        return np.asarray(d).astype(np.float32)
    if s_to in ("i32", "u32"):
        if s_from == "f32":
            return _f2i(d, s_to)
        return np.asarray(d).astype(np.int64).astype(_NP[s_to])
    if s_to == "bool":
        return np.asarray(d) != 0
    raise WgslError(f"{s_from} -> {s_to}")


def unorm8_store(v: np.ndarray, pins: Pins = PINS) -> np.ndarray:
    """rgba8unorm store of f32 values: clamp to [0, 1] (NaN -> 0), scale by
    255 in f32, round (half to even, or half up)."""
    v = np.asarray(v, dtype=np.float32)
    with np.errstate(invalid="ignore"):
        c = np.where(np.isnan(v), F32(0.0), np.clip(v, F32(0.0), F32(1.0))).astype(np.float32)
        s = (c * F32(255.0)).astype(np.float32)
        r = np.rint(s) if pins.store_round == "half_even" else np.floor(s + F32(0.5))
    return r.astype(np.uint8)
