"""Every ``profiles/...`` evidence file cited by the code and docs exists.

Scans the repo's own sources and docs (not the judge's VERDICT/ADVICE, which may name files to be
produced). A citation is a path under profiles/ with a file extension; a trailing ``*`` / ``{a,b}``
glob or brace form is expanded against the tree."""

import glob
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP = {"VERDICT.md", "ADVICE.md", "PAPERS.md", "SNIPPETS.md", "SURVEY.md"}
CITE = re.compile(r"profiles/[A-Za-z0-9_.\-/{},*]+")


def _files():
    for pat in ("*.py", "*.md", "**/*.py", "**/*.md", "csrc/**/*.hip", "csrc/**/*.cpp", "csrc/**/*.h", "scripts/*.sh"):
        for p in glob.glob(os.path.join(REPO, pat), recursive=True):
            rel = os.path.relpath(p, REPO)
            if os.path.basename(p) in SKIP or rel.startswith(("gpurun_out", ".git")) or "/_snapshots/" in p:
                continue
            yield p


def _expand(c: str) -> list[str]:
    m = re.search(r"\{([^}]*)\}", c)
    if not m:
        return [c]
    out = []
    for alt in m.group(1).split(","):
        out += _expand(c[: m.start()] + alt + c[m.end():])
    return out


def test_profile_citations_exist():
    missing = set()
    for p in set(_files()):
        text = open(p, encoding="utf-8", errors="replace").read()
        for c in CITE.findall(text):
            c = c.rstrip(".,)")
            for path in _expand(c):
                path = path.rstrip(".,)")
                if not re.search(r"\.[A-Za-z]{1,5}$", path) and "*" not in path:
                    continue  # a directory or a prefix, not a file citation
                full = os.path.join(REPO, path)
                if "*" in path:
                    if not glob.glob(full):
                        missing.add((os.path.relpath(p, REPO), path))
                elif not os.path.exists(full):
                    missing.add((os.path.relpath(p, REPO), path))
    assert not missing, sorted(missing)
