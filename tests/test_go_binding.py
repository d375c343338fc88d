"""CPU checks of the cgo binding (go/gpu/wvgpu.go) against the C ABI header.

There is no Go toolchain in this image, so the binding cannot be compiled
here; these tests pin what can drift silently: every C.wvg_* call names an
entry point of include/wvgpu.h with the header's argument count, every
constant it reads is a header macro, the binding covers the header (test
helpers aside), and a non-nil empty AllowList returns no results instead of
reaching the library as "no filter" (V/flat/index.go:423-427)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wvgpu.h")
GO_DIR = os.path.join(ROOT, "go", "gpu")
# bench / test helpers with no Go caller
NOT_BOUND = {"wvg_corpus_fill_synthetic", "wvg_synthetic_rows", "wvg_multi_corpus_fill_synthetic"}  # test helpers


def header_prototypes():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for name, params in re.findall(r"\b(wvg_[a-z0-9_]+)\s*\(([^()]*)\)\s*;", src):
        params = params.strip()
        out[name] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def header_macros():
    return set(re.findall(r"#define\s+(WVG_[A-Z0-9_]+)", open(HEADER).read()))


def go_source(name="wvgpu.go"):
    return open(os.path.join(GO_DIR, name)).read()


def strip_go_comments(src):
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def go_calls(src):
    """(name, argument count, line) of every C.wvg_*( ... ) call."""
    body = strip_go_comments(src)
    out = []
    for m in re.finditer(r"\bC\.(wvg_[a-z0-9_]+)\s*\(", body):
        i, depth, commas, nonblank = m.end(), 1, 0, False
        while depth:
            ch = body[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == "," and depth == 1:
                commas += 1
            elif ch == '"':
                i = body.index('"', i + 1)
            if depth and not ch.isspace():
                nonblank = True
            i += 1
        out.append((m.group(1), commas + 1 if nonblank else 0, body.count("\n", 0, m.start()) + 1))
    return out


def test_go_binding_exists_with_build_tag():
    src = go_source()
    assert src.startswith("//go:build rocm\n")
    assert 'import "C"' in src and '#include "wvgpu.h"' in src


def test_every_cgo_call_matches_the_header():
    protos = header_prototypes()
    calls = go_calls(go_source())
    assert len(calls) >= 40
    bad = [(n, a, ln, protos.get(n)) for n, a, ln in calls if protos.get(n) != a]
    assert not bad, f"C.wvg_* calls that do not match include/wvgpu.h (name, args, line, header args): {bad}"


def test_cgo_constants_and_types_exist():
    src = strip_go_comments(go_source())
    macros = header_macros()
    used = set(re.findall(r"\bC\.(WVG_[A-Z0-9_]+)", src))
    assert used and used <= macros, used - macros
    # the option struct's fields as the header declares them
    fields = set(re.findall(r"\bopt\.([a-z_]+)|\bo\.([a-z_]+)", src))
    fields = {a or b for a, b in fields}
    hdr = open(HEADER).read()
    for f in fields:
        assert re.search(r"\b%s;" % f, hdr), f


def test_binding_covers_the_header():
    bound = {n for n, _, _ in go_calls(go_source())}
    missing = set(header_prototypes()) - bound - NOT_BOUND
    assert not missing, sorted(missing)


def test_empty_allow_list_is_not_a_nil_filter():
    """Every search that takes an AllowList goes through allowBitmap, which
    reports a non-nil empty list (IsEmpty) so the caller returns without a
    call; a nil list is the only "no filter"."""
    src = strip_go_comments(go_source())
    fn = re.search(r"func allowBitmap\(allow helpers\.AllowList\) \(words \[\]uint64, ok bool\) \{(.*?)\n\}", src,
                   re.S).group(1)
    assert re.search(r"if allow == nil \{\s*return nil, true", fn)
    assert re.search(r"if allow\.IsEmpty\(\) \{\s*return nil, false", fn)
    # every Go function taking a helpers.AllowList converts it and honours ok == false before any call
    for m in re.finditer(r"func \([^)]*\) (\w+)\(([^)]*)\)[^{]*\{", src):
        if "helpers.AllowList" not in m.group(2):
            continue
        body = src[m.end():src.index("\n}\n", m.end())]
        if m.group(1) == "Search":  # delegates to SearchBatch
            assert "x.SearchBatch(" in body
            continue
        conv = body.find("allowBitmap(allow)")
        first_call = body.find("C.wvg_")
        assert 0 <= conv < first_call, m.group(1)
        assert re.search(r"if !ok \{\s*return", body[conv:first_call]), m.group(1)
        assert "u64p(words)" in body[first_call:], m.group(1)
