"""The timing-only A/B variants of tools/ab_variants.py still apply to the product sources.

Every substitution's `old` text must occur exactly once in its file (the rule build() enforces
at build time), so a recorded A/B under profiles/ can be re-run on the current sources.  CPU
only: no build, no GPU."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _variants():
    spec = importlib.util.spec_from_file_location("ab_variants", os.path.join(REPO, "tools", "ab_variants.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_every_variant_applies_once():
    mod = _variants()
    assert "head" in mod.VARIANTS and mod.VARIANTS["head"] == []
    for name, subs in mod.VARIANTS.items():
        texts = {}
        for fname, old, new in subs:
            path = os.path.join(mod.CSRC, fname)
            src = texts.setdefault(fname, open(path).read())
            assert src.count(old) == 1, f"variant {name}: text occurs {src.count(old)} times in {fname}"
            assert old != new, f"variant {name}: a substitution changes nothing"
            # later substitutions of the same variant see the earlier ones
            texts[fname] = src.replace(old, new)
