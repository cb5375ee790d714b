"""Configuration hygiene: every ``CS336_*`` environment variable the library, the
native code and ``bench.py`` read is documented in README's environment table; every ``CS336_*``
build define the kernels test is in README's build-switch table; and no kernel source carries a
probe switch that produces wrong results (those live as patches in ``scripts/variants/``), nor a
knob that was measured, found not to help and dropped."""

import pathlib
import re

REPO = pathlib.Path(__file__).resolve().parents[1]
CODE = [REPO / "cs336_systems", REPO / "csrc", REPO / "bench.py", REPO / "__graft_entry__.py"]


def _files():
    for root in CODE:
        if root.is_file():
            yield root
        else:
            yield from (f for f in root.rglob("*") if f.suffix in (".py", ".cpp", ".hip", ".h"))


def _readme():
    return (REPO / "README.md").read_text()


def test_every_env_switch_is_documented():
    names = set()
    for f in _files():
        names |= set(re.findall(r"[\"'](CS336_[A-Z0-9_]+)[\"']", f.read_text(errors="ignore")))
    table = "\n".join(line for line in _readme().splitlines() if line.startswith("| `CS336_"))
    missing = sorted(n for n in names if f"`{n}" not in table and f", `{n}" not in table and f"{n}=" not in table)
    assert not missing, f"undocumented CS336_* environment switches: {missing}"


def test_every_build_define_is_documented():
    defines = set()
    for f in _files():
        defines |= set(re.findall(r"#\s*if(?:n?def)?\s+(?:defined\()?\s*(CS336_[A-Z0-9_]+)", f.read_text(errors="ignore")))
    readme = _readme()
    missing = sorted(d for d in defines if f"`{d}" not in readme)
    assert not missing, f"undocumented CS336_* build defines: {missing}"


def test_no_wrong_result_probe_in_kernels():
    bad = []
    for f in (REPO / "csrc").rglob("*"):
        if f.suffix not in (".hip", ".h", ".cpp"):
            continue
        for i, line in enumerate(f.read_text(errors="ignore").splitlines(), 1):
            if re.match(r"\s*#\s*if", line) and "wrong" in line.lower():
                bad.append(f"{f.relative_to(REPO)}:{i}")
    assert not bad, bad


# Measured-and-dropped knobs: once an A/B rejects a variant, its switch leaves the shipped sources
# (the measurement stays in profiles/). Patterns of every such knob retired so far.
RETIRED_KNOBS = [
    r"\bstg_\w+",                # gemm8 first-round stagger (profiles/r5_gemm8_epilogue.md)
    r"\bset_stagger\b",
    r"gemm8_stagger",
    r"G8_STAGGER",                # round-3 form of the same (profiles/r3_gemm8_stagger_ab.md)
    r"G8_PERSIST",                # persistent gemm8 (profiles/r3_gemm8_persistent_ab.md, r5_step_clocks.md)
    r"G8_NO_EPI",
    r"G8_ABL_",                   # epilogue ablation builds (profiles/r5_gemm8_epilogue.md)
    r"PersistentGrads|grad[-_]buffers",  # 1-GPU persistent gradient views (profiles/r6_ddp_world1.md)
]


def test_no_retired_knob_in_sources():
    bad = []
    for f in _files():
        text = f.read_text(errors="ignore")
        for pat in RETIRED_KNOBS:
            for m in re.finditer(pat, text):
                line = text.count("\n", 0, m.start()) + 1
                bad.append(f"{f.relative_to(REPO)}:{line}: {m.group(0)}")
    assert not bad, f"measured-and-dropped knobs still in the sources: {bad}"
