"""Lexical and call-shape checks of the Rust crate (chunky-bits_amd/rust/chunky-ec-sys), which no
cargo in this image compiles: every source file tokenizes (comments, strings, raw strings, char
literals vs lifetimes) with balanced brackets, and every call of a method the crate defines --
`self.f(..)` in an impl block and `self.multi.f(..)` / `self.rp.f(..)` on the crate's own
wrappers -- names a method that exists with that many arguments, and so does every call of the
crate's free and associated functions; every `self.field` names a field of its struct; and every
variable a function body uses is declared in that function.  A renamed method, a call left with
the old argument list (as an FFI wrapper grows a parameter) or a variable an edit left behind
fails here.""" 
import os
import re

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "chunky-bits_amd",
                   "rust", "chunky-ec-sys", "src")
FILES = sorted(f for f in os.listdir(SRC) if f.endswith(".rs"))


def tokens(src):
    """(kind, text, line) for Rust source: kinds ident, punct, str, char, num, lifetime."""
    out, i, line, n = [], 0, 1, len(src)
    while i < n:
        c = src[i]
        if c == "\n":
            line += 1
            i += 1
        elif c.isspace():
            i += 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):  # nested block comments
            depth, j = 1, i + 2
            while depth and j < n:
                if src.startswith("/*", j):
                    depth, j = depth + 1, j + 2
                elif src.startswith("*/", j):
                    depth, j = depth - 1, j + 2
                else:
                    j += 1
            assert depth == 0, f"unterminated block comment from line {line}"
            line += src.count("\n", i, j)
            i = j
        elif re.match(r'b?r#*"', src[i:i + 8]):  # raw (byte) string
            m = re.match(r'(b?r)(#*)"', src[i:])
            end = '"' + m.group(2)
            j = src.find(end, i + len(m.group(0)))
            assert j >= 0, f"unterminated raw string at line {line}"
            j += len(end)
            out.append(("str", src[i:j], line))
            line += src.count("\n", i, j)
            i = j
        elif c == '"' or src.startswith('b"', i):
            j = i + (2 if c == "b" else 1)
            while j < n and src[j] != '"':
                j += 2 if src[j] == "\\" else 1
            assert j < n, f"unterminated string at line {line}"
            out.append(("str", src[i:j + 1], line))
            line += src.count("\n", i, j)
            i = j + 1
        elif c == "'" or src.startswith("b'", i):
            k = i + (1 if c == "b" else 0)
            m = re.match(r"'(\\(?:u\{[0-9a-fA-F]+\}|x[0-9a-fA-F]{2}|.)|[^\\'])'", src[k:])
            if m:
                out.append(("char", src[i:k + len(m.group(0))], line))
                i = k + len(m.group(0))
            else:
                m = re.match(r"'[A-Za-z_][A-Za-z0-9_]*", src[i:])
                assert m, f"stray quote at line {line}"
                out.append(("lifetime", m.group(0), line))
                i += len(m.group(0))
        elif c.isalpha() or c == "_":
            m = re.match(r"[A-Za-z_][A-Za-z0-9_]*", src[i:])
            out.append(("ident", m.group(0), line))
            i += len(m.group(0))
        elif c.isdigit():
            m = re.match(r"[0-9][0-9a-zA-Z_]*(\.[0-9][0-9_]*)?([eE][+-]?[0-9]+)?[a-z0-9]*", src[i:])
            out.append(("num", m.group(0), line))
            i += len(m.group(0))
        else:
            two = src[i:i + 2]
            if two in ("::", "->", "=>", "==", "!=", "<=", ">=", "&&", "||", "..", "+=", "-=",
                       "*=", "|=", "&=", "^=", "<<", ">>"):
                out.append(("punct", two, line))
                i += 2
            else:
                out.append(("punct", c, line))
                i += 1
    return out


def _read(f):
    return open(os.path.join(SRC, f)).read()


@pytest.mark.parametrize("name", FILES)
def test_rust_source_tokenizes_with_balanced_brackets(name):
    stack = []
    pairs = {")": "(", "]": "[", "}": "{"}
    for kind, text, line in tokens(_read(name)):
        if kind != "punct":
            continue
        if text in "([{":
            stack.append((text, line))
        elif text in ")]}":
            assert stack, f"{name}:{line}: unmatched {text}"
            opened, at = stack.pop()
            assert opened == pairs[text], f"{name}:{line}: {text} closes {opened} of line {at}"
    assert not stack, f"{name}: unclosed {stack[-1]}"


def _group(toks, i):
    """Index just past the bracket group opening at toks[i]."""
    depth = 0
    for j in range(i, len(toks)):
        t = toks[j][1] if toks[j][0] == "punct" else None
        if t in ("(", "[", "{"):
            depth += 1
        elif t in (")", "]", "}"):
            depth -= 1
            if depth == 0:
                return j + 1
    raise AssertionError("unbalanced")


def _args(toks, i):
    """Number of top-level arguments of the call whose '(' is toks[i] (closures' |a, b| skipped)."""
    end = _group(toks, i)
    inner = toks[i + 1:end - 1]
    if not inner:
        return 0
    count, j, at_start = 1, 0, True
    while j < len(inner):
        kind, t, _ = inner[j]
        if kind == "punct" and t in ("(", "[", "{"):
            j = i + 1 + j
            j = _group(toks, j) - (i + 1)
            at_start = False
            continue
        if kind == "punct" and t == "|" and at_start:  # closure parameters
            j += 1
            while not (inner[j][0] == "punct" and inner[j][1] == "|"):
                j += 1
        elif kind == "punct" and t == "||" and at_start:
            pass
        elif kind == "ident" and t == "move" and at_start:
            j += 1
            continue
        elif kind == "punct" and t == ",":
            if j + 1 < len(inner):
                count += 1
            at_start = True
            j += 1
            continue
        at_start = False
        j += 1
    return count


def _methods(src):
    """{impl type: {name: parameter counts}} of every fn with a self receiver (self excluded),
    {"Type::": ...} of the associated functions and {"": ...} of the free functions."""
    toks = tokens(src)
    out = {}
    impl = None
    depth, impl_depth = 0, None
    for i, (kind, t, _) in enumerate(toks):
        if kind == "punct" and t == "{":
            depth += 1
        elif kind == "punct" and t == "}":
            depth -= 1
            if impl_depth is not None and depth < impl_depth:
                impl, impl_depth = None, None
        elif kind == "ident" and t == "impl" and impl is None:
            j = i + 1
            if toks[j][1] == "<":  # impl<T>
                while toks[j][1] != ">":
                    j += 1
                j += 1
            name = toks[j][1]
            # `impl Trait for Type`
            k = j
            while toks[k][1] != "{":
                if toks[k][1] == "for":
                    name = toks[k + 1][1]
                k += 1
            impl, impl_depth = name, depth + 1
        elif kind == "ident" and t == "fn" and impl is not None:
            name = toks[i + 1][1]
            j = i + 2
            if toks[j][1] == "<":
                lvl = 0
                while True:
                    lvl += {"<": 1, ">": -1, ">>": -2, "<<": 2}.get(toks[j][1], 0)
                    j += 1
                    if lvl <= 0:
                        break
            assert toks[j][1] == "(", (name, toks[j])
            n = _args(toks, j)
            has_self = any(x[1] == "self" for x in toks[j + 1:_group(toks, j)][:3])
            if has_self:
                out.setdefault(impl, {}).setdefault(name, set()).add(n - 1)
            else:  # an associated function: Type::name(..)
                out.setdefault(impl + "::", {}).setdefault(name, set()).add(n)
        elif kind == "ident" and t == "fn" and impl is None and toks[i + 2][1] in ("(", "<"):
            j = i + 2
            while toks[j][1] != "(":
                j += 1
            out.setdefault("", {}).setdefault(toks[i + 1][1], set()).add(_args(toks, j))
    return out


def test_method_calls_name_existing_methods_with_their_arity():
    defs = {}
    for f in FILES:
        for impl, ms in _methods(_read(f)).items():
            for name, ns in ms.items():
                defs.setdefault(impl, {}).setdefault(name, set()).update(ns)
    assert "Multi" in defs and "BatchReader" in defs
    receivers = {"multi": "Multi", "rp": "ReadPipeline"}
    checked = 0
    for f in FILES:
        toks = tokens(_read(f))
        # the impl type around each position
        for i in range(len(toks) - 4):
            if toks[i][1] != "self" or toks[i + 1][1] != ".":
                continue
            if toks[i + 3][1] == "(" and toks[i + 2][0] == "ident":
                owner, name, paren = None, toks[i + 2][1], i + 3
                # self.f(..): a method of whichever impl defines it in this crate
                cands = [t for t, ms in defs.items() if name in ms]
                if not cands:
                    continue  # a std trait method (clone, iter, ...)
                n = _args(toks, paren)
                assert any(n in defs[t][name] for t in cands), \
                    f"{f}:{toks[i][2]}: self.{name}() with {n} args; defined {[defs[t][name] for t in cands]}"
                checked += 1
            elif (toks[i + 2][1] in receivers and toks[i + 3][1] == "." and toks[i + 5][1] == "("
                  if i + 5 < len(toks) else False):
                owner, name = receivers[toks[i + 2][1]], toks[i + 4][1]
                if owner not in defs:
                    continue
                assert name in defs[owner], f"{f}:{toks[i][2]}: {owner} has no method {name}"
                n = _args(toks, i + 5)
                assert n in defs[owner][name], \
                    f"{f}:{toks[i][2]}: self.{toks[i + 2][1]}.{name}() with {n} args, defined {defs[owner][name]}"
                checked += 1
    assert checked > 50


def test_function_calls_match_the_crates_definitions():
    """Free functions (`draw_order(..)`) and associated functions (`Multi::new(..)`) of the crate
    are called with as many arguments as they take."""
    defs = {}
    for f in FILES:
        for impl, ms in _methods(_read(f)).items():
            for name, ns in ms.items():
                defs.setdefault(impl, {}).setdefault(name, set()).update(ns)
    free = defs.get("", {})
    assert "draw_order" in free or "next_copy" in free or len(free) > 3
    checked = 0
    for f in FILES:
        toks = tokens(_read(f))
        for i in range(1, len(toks) - 1):
            kind, name, line = toks[i]
            if kind != "ident" or toks[i + 1][1] != "(" or toks[i - 1][1] in ("fn", ".", "!"):
                continue
            if toks[i - 1][1] == "::":
                owner = toks[i - 2][1] + "::"
                if owner == "Self::":
                    continue  # resolved by the impl in scope; the method check covers self calls
                if owner in defs and name in defs[owner]:
                    n = _args(toks, i + 1)
                    assert n in defs[owner][name], f"{f}:{line}: {owner}{name}() with {n} args"
                    checked += 1
            elif name in free:
                n = _args(toks, i + 1)
                assert n in free[name], f"{f}:{line}: {name}() with {n} args, defined {free[name]}"
                checked += 1
    assert checked > 20


def _struct_fields(toks):
    """{struct name: field names} of the named-field structs."""
    out = {}
    for i, (kind, t, _) in enumerate(toks):
        if kind == "ident" and t == "struct":
            name = toks[i + 1][1]
            j = i + 2
            while toks[j][1] not in ("{", ";", "("):
                j += 1
            if toks[j][1] != "{":
                continue
            end = _group(toks, j)
            fields, depth = set(), 0
            for k in range(j + 1, end - 1):
                x = toks[k][1]
                if x in ("(", "[", "{", "<"):
                    depth += 1
                elif x in (")", "]", "}", ">"):
                    depth -= 1
                elif x == ">>":
                    depth -= 2
                elif (depth == 0 and toks[k][0] == "ident" and toks[k + 1][1] == ":"
                      and toks[k - 1][1] in ("{", ",", "pub", ")")):
                    fields.add(x)
            out[name] = fields
    return out


def test_self_fields_exist_in_their_struct():
    """Inside `impl Type`, every `self.name` that is not a call names a field of struct Type."""
    fields = {}
    for f in FILES:
        fields.update(_struct_fields(tokens(_read(f))))
    assert "BatchReader" in fields and "windows" in fields["BatchReader"]
    checked = 0
    for f in FILES:
        toks = tokens(_read(f))
        impl, depth, impl_depth = None, 0, None
        for i, (kind, t, line) in enumerate(toks):
            if kind == "punct" and t == "{":
                depth += 1
            elif kind == "punct" and t == "}":
                depth -= 1
                if impl_depth is not None and depth < impl_depth:
                    impl, impl_depth = None, None
            elif kind == "ident" and t == "impl" and impl is None:
                j = i + 1
                if toks[j][1] == "<":
                    while toks[j][1] != ">":
                        j += 1
                    j += 1
                name, k = toks[j][1], j
                while toks[k][1] != "{":
                    if toks[k][1] == "for":
                        name = toks[k + 1][1]
                    k += 1
                impl, impl_depth = name, depth + 1
            elif (impl in fields and kind == "ident" and t == "self" and toks[i + 1][1] == "."
                  and toks[i + 2][0] == "ident" and toks[i + 3][1] not in ("(", "::")):
                name = toks[i + 2][1]
                assert name in fields[impl], f"{f}:{line}: {impl} has no field {name}"
                checked += 1
    assert checked > 100


# ---- per-function scope: every variable a function body uses is declared in it ----------------
KW = set("""as break const continue crate else enum extern false fn for if impl in let loop match mod move mut
pub ref return self Self static struct super trait true type unsafe use where while async await dyn box
u8 u16 u32 u64 u128 usize i8 i16 i32 i64 i128 isize f32 f64 bool char str c_int c_uint c_char c_void
c_long c_ulong""".split())

def _module_names(toks):
    names = set()
    for i, (k, x, _) in enumerate(toks):
        if k == 'ident' and x in ('fn', 'const', 'static', 'mod', 'struct', 'enum', 'type', 'trait') and i + 1 < len(toks):
            names.add(toks[i + 1][1])
        if k == 'ident' and x == 'use':
            j = i + 1
            while toks[j][1] != ';':
                if toks[j][0] == 'ident':
                    names.add(toks[j][1])
                j += 1
    return names

def _pattern_idents(toks, a, b, closure=False):
    out = set()
    for j in range(a, b):
        k, x, _ = toks[j]
        if k == 'ident' and x not in KW and not x[0].isupper():
            nxt = toks[j + 1][1] if j + 1 < len(toks) else ''
            prv = toks[j - 1][1]
            if nxt in ('(', '::', '{') or prv in ('::', '.'):
                continue
            if nxt == ':' and prv in ('{', ',') and not closure:  # field: pattern
                continue
            out.add(x)
    return out

def _undeclared_uses(fname):
    src = _read(fname)
    toks = tokens(src)
    mods = _module_names(toks)
    problems = []
    i = 0
    while i < len(toks):
        if toks[i][1] == 'fn' and toks[i][0] == 'ident' and i + 1 < len(toks) and toks[i + 1][0] == 'ident':
            name = toks[i + 1][1]
            j = i + 2
            while toks[j][1] != '(':
                j += 1
            pend = _group(toks, j)
            declared = set()
            # params: ident before ':' at depth 1 of the param list, or self
            depth = 0
            for q in range(j, pend):
                x = toks[q][1]
                if x in '([{':
                    depth += 1
                elif x in ')]}':
                    depth -= 1
                elif depth == 1 and toks[q][0] == 'ident' and toks[q + 1][1] == ':' :
                    declared.add(x)
            b = pend
            while b < len(toks) and toks[b][1] not in ('{', ';'):
                b += 1
            if toks[b][1] == ';':
                i = b
                continue
            bend = _group(toks, b)
            body = range(b, bend)
            # declarations in the body
            for q in body:
                k, x, _ = toks[q]
                if x == 'let':
                    r = q + 1
                    depth = 0
                    while not (depth == 0 and toks[r][1] in ('=', ';', ':')):
                        if toks[r][1] in '([{':
                            depth += 1
                        elif toks[r][1] in ')]}':
                            depth -= 1
                        r += 1
                    declared |= _pattern_idents(toks, q + 1, r)
                elif x == 'for' and toks[q - 1][1] != '<':
                    r = q + 1
                    while toks[r][1] != 'in':
                        r += 1
                    declared |= _pattern_idents(toks, q + 1, r)
                elif x in ('|', '||') and k == 'punct' and x == '|':
                    # closure params: | ... | when preceded by ( , = move or start of arg
                    prv = toks[q - 1][1]
                    if prv in ('(', ',', '=', 'move', '{', ';', 'return') :
                        r = q + 1
                        while toks[r][1] != '|':
                            r += 1
                        declared |= _pattern_idents(toks, q + 1, r, closure=True)
                elif x == '=>':
                    # match arm pattern: back to the previous ',' or '{' at this depth
                    r = q - 1
                    depth = 0
                    while True:
                        y = toks[r][1]
                        if y in ')]}':
                            depth += 1
                        elif y in '([{':
                            if depth == 0:
                                break
                            depth -= 1
                        elif y == ',' and depth == 0:
                            break
                        r -= 1
                    declared |= _pattern_idents(toks, r + 1, q)
            # uses
            for q in body:
                k, x, line = toks[q]
                if k != 'ident' or x in KW or x[0].isupper() or x in declared or x in mods:
                    continue
                prv, nxt = toks[q - 1][1], toks[q + 1][1]
                if prv in ('.', '::', "'") or nxt in ('(', '!', '::'):
                    continue
                if nxt == ':' and prv in ('{', ','):  # struct literal field
                    continue
                if prv == '<' or nxt == '>' :  # generic args / lifetimes-ish
                    continue
                problems.append((fname, line, name, x))
            i = bend
            continue
        i += 1
    return problems



def test_function_bodies_use_only_declared_names():
    """Every lower-case name a function body uses as a value is declared in that function (a
    parameter, a `let` / `for` / `if let` / match-arm / closure pattern) or at module level (a
    fn, const, static or import): a variable left behind by an edit (used in a function that
    never binds it) fails here.  Conservative: calls, paths, fields and types are not checked."""
    problems = [p for f in FILES for p in _undeclared_uses(f)]
    assert not problems, problems


# ---- names: imports from the crate root exist there, and every type-like name resolves ---------
_PRELUDE = set("""Vec Option Some None Result Ok Err String Box Self FnMut Fn FnOnce Copy Clone Debug
PartialEq Eq Default Drop Send Sync Sized Iterator IntoIterator From Into AsRef AsMut ToString
Display Hash Ord PartialOrd VecDeque HashMap BTreeMap Cow Arc Rc Mutex Duration Instant""".split())


def _defined(toks):
    """Names a file defines at any level: items, and the variants of its enums."""
    out = set()
    for i, (k, x, _) in enumerate(toks):
        if k == "ident" and x in ("struct", "enum", "type", "trait", "fn", "const", "static", "mod",
                                  "union"):
            out.add(toks[i + 1][1])
        if k == "ident" and x == "enum":
            j = i + 2
            while toks[j][1] != "{":
                j += 1
            end, depth = _group(toks, j), 0
            for q in range(j + 1, end - 1):
                y = toks[q][1]
                if y in "([{":
                    depth += 1
                elif y in ")]}":
                    depth -= 1
                elif depth == 0 and toks[q][0] == "ident" and toks[q - 1][1] in ("{", ","):
                    out.add(y)
    return out


def _imported(toks):
    out = set()
    for i, (k, x, _) in enumerate(toks):
        if k == "ident" and x == "use":
            j = i + 1
            while toks[j][1] != ";":
                if toks[j][0] == "ident":
                    out.add(toks[j][1])
                j += 1
    return out


def test_names_resolve():
    """`use crate::{..}` names and `crate::name` paths exist at the crate root (lib.rs defines or
    re-exports them), and every CamelCase name a file uses unqualified is defined in it, imported,
    or in the std prelude: a type renamed in one file and not the other fails here."""
    lib = tokens(_read("lib.rs"))
    root = _defined(lib) | _imported(lib)
    problems = []
    for f in FILES:
        toks = tokens(_read(f))
        known = _defined(toks) | _imported(toks) | _PRELUDE | (root if f == "lib.rs" else set())
        for i, (k, x, line) in enumerate(toks):
            if x == "use" and toks[i + 1][1] == "crate":
                j = i + 2
                while toks[j][1] != ";":
                    if toks[j][0] == "ident" and toks[j][1] != "self" and toks[j][1] not in root:
                        problems.append((f, line, "use crate::" + toks[j][1]))
                    j += 1
            if (x == "crate" and toks[i + 1][1] == "::" and toks[i + 2][0] == "ident"
                    and toks[i + 2][1] not in root | {"sys", "batch"}):
                problems.append((f, line, "crate::" + toks[i + 2][1]))
            if (k == "ident" and x[0].isupper() and not x.isupper() and toks[i - 1][1] not in ("::", ".")
                    and x not in known):
                problems.append((f, line, x))
    assert not problems, problems


# method names the standard library also has: calls of these on other receivers are not checked
_STD_METHODS = set("""len iter iter_mut read write get get_mut push insert new clone as_ptr as_mut_ptr map
take skip filter collect chunks copy_from_slice fill extend resize contains min max wait drain flush
run encode from into sum count any all first last is_empty unwrap expect ok err map_err and_then find
position to_vec as_slice swap remove pop push_back pop_front sort dedup retain split_at chain zip
enumerate rev windows step_by next send recv lock join spawn fmt eq cmp hash default drop as_ref
as_mut borrow entry with_capacity reserve truncate clear set query stats release carry_release verify
resilver""".split())


def test_crate_method_calls_on_other_receivers_match_arity():
    """`x.f(..)` where f is a method only this crate defines (not a std method name): called with
    as many arguments as a definition takes, whatever the receiver."""
    defs = {}
    for f in FILES:
        for impl, ms in _methods(_read(f)).items():
            if impl.endswith("::") or impl == "":
                continue
            for name, ns in ms.items():
                defs.setdefault(name, set()).update(ns)
    own = {n: ns for n, ns in defs.items() if n not in _STD_METHODS}
    problems, checked = [], 0
    for f in FILES:
        toks = tokens(_read(f))
        for i in range(1, len(toks) - 2):
            if (toks[i][1] == "." and toks[i + 1][0] == "ident" and toks[i + 2][1] == "("
                    and toks[i - 1][1] != "self" and toks[i + 1][1] in own):
                n = _args(toks, i + 2)
                checked += 1
                if n not in own[toks[i + 1][1]]:
                    problems.append((f, toks[i][2], toks[i + 1][1], n))
    assert checked >= 10 and not problems, problems
