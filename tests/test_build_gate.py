"""The rebuild gate of vcf_amd/_build.py sees every header a source includes.

VERDICT r05 weak item 7: HEADERS once omitted vcf_dwt_lift.h, so an edit to
the lifting kernels did not trigger a rebuild.  needs_rebuild() now scans the
sources' includes transitively; these tests pin that.
"""
import os

from vcf_amd import _build


def _all_local_headers():
    seen, todo = set(), list(_build.SOURCES + _build.AB_SOURCES)
    out = set()
    while todo:
        rel = todo.pop()
        path = os.path.join(_build.CSRC, rel)
        if path in seen or not os.path.exists(path):
            continue
        seen.add(path)
        for name in _build.local_includes(path):
            if os.path.exists(os.path.join(_build.CSRC, name)):
                out.add(name)
                todo.append(name)
    return out


def test_every_included_csrc_header_is_listed():
    # (ab/vcf_inflate_wincheck.hip includes a whole .hip source, which is in SOURCES)
    headers = {h for h in _all_local_headers() if h.endswith(".h")}
    missing = headers - set(_build.HEADERS)
    assert not missing, f"headers included by sources but not in HEADERS: {sorted(missing)}"


def test_deps_mtime_is_transitive():
    # vcf_dwt.hip includes vcf_dwt_lift.h
    lift = os.path.join(_build.CSRC, "vcf_dwt_lift.h")
    assert "vcf_dwt_lift.h" in _build.local_includes(os.path.join(_build.CSRC, "vcf_dwt.hip"))
    assert _build.deps_mtime("vcf_dwt.hip") >= os.path.getmtime(lift)


def test_touching_a_header_triggers_rebuild(monkeypatch):
    if not (os.path.exists(_build.LIB) and os.path.exists(_build.AB_LIB)):
        assert _build.needs_rebuild()
        return
    t = min(os.path.getmtime(_build.LIB), os.path.getmtime(_build.AB_LIB))
    lift = os.path.join(_build.CSRC, "vcf_dwt_lift.h")
    real = os.path.getmtime

    def fake(path):
        if os.path.abspath(path) == lift:
            return t + 10.0
        return real(path)

    monkeypatch.setattr(os.path, "getmtime", fake)
    assert _build.needs_rebuild()
