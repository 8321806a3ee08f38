"""CPU-side checks of the C ABI: the gfx950 library builds, loads, and exports every symbol that
include/gbv.h declares.  No compute calls (there is no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "gbv.h")).read()
    return sorted(set(re.findall(r"\b(gbv_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding():
    from lodestar_amd import _native
    assert sorted(_native.EXPORTED_SYMBOLS) == declared_symbols()


def test_library_exports_all_symbols():
    from lodestar_amd import build
    build.build()
    lib = ctypes.CDLL(build.LIB)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object():
    from lodestar_amd import build
    data = open(build.LIB, "rb").read()
    assert b"gfx950" in data


def test_no_oracle_import_in_product():
    """The product never imports or includes anything under oracle/ (test infrastructure only)."""
    import ast
    for dirpath, _, files in os.walk(os.path.join(ROOT, "lodestar_amd")):
        for f in files:
            path = os.path.join(dirpath, f)
            if f.endswith(".py"):
                tree = ast.parse(open(path).read())
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        assert not any(a.name.split(".")[0] == "oracle" for a in node.names), path
                    elif isinstance(node, ast.ImportFrom):
                        assert (node.module or "").split(".")[0] != "oracle", path
            elif f.endswith((".h", ".hip", ".cpp")):
                assert "oracle/" not in open(path).read(), path


def test_tuning_names_documented():
    """Every gbv_tune name the library accepts (gbv.hip tuning_set's table and the per-context names in
    gbv_tune) is listed in include/gbv.h's gbv_tune comment, and every listed name is accepted."""
    import re
    src = open(os.path.join(ROOT, "lodestar_amd", "csrc", "gbv.hip")).read()
    table = src[src.index("bool tuning_set("):]
    table = table[:table.index("};")]
    process_wide = set(re.findall(r'\{"([a-z_0-9]+)", &g_tuning\.', table))
    per_ctx = set(re.findall(r'!strcmp\(name, "([a-z_0-9]+)"\)', src[src.index("int gbv_tune("):]))
    hdr = open(os.path.join(ROOT, "include", "gbv.h")).read()
    doc = hdr[:hdr.index("int gbv_tune(")]
    doc = doc[doc.rindex("/*"):]
    listed = set(re.findall(r'"([a-z_0-9]+)"', doc))
    assert process_wide and per_ctx
    assert process_wide | per_ctx == listed, (sorted((process_wide | per_ctx) - listed), sorted(listed - (process_wide | per_ctx)))
