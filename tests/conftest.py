import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "fuzzy-aho-corasick-rs_amd")
for p in (REPO, PKG_DIR, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# The library honours its FAC_* tuning / test knobs only in diagnostics mode (fac.h); the tests use
# them (monkeypatch.setenv) to force kernel paths.
os.environ["FAC_DIAGNOSTICS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU; run on the GPU box")


def _oracle_factory(builder, patterns):
    from oracle_harness import OracleEngine
    return OracleEngine(builder, patterns)


def _gpu_factory(builder, patterns):
    return builder.build(patterns)


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def make_engine(request):
    """Build an engine from a FuzzyAhoCorasickBuilder on the CPU oracle or on the GPU."""
    return _oracle_factory if request.param == "oracle" else _gpu_factory


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def make_replacer(request):
    def f(builder, pairs):
        from fuzzy_aho_corasick import FuzzyReplacer, Pattern
        from oracle_harness import OracleReplacer
        pats = [Pattern.from_(p) for p, _ in pairs]
        repl = [r for _, r in pairs]
        if request.param == "oracle":
            return OracleReplacer(_oracle_factory(builder, pats), repl)
        return FuzzyReplacer(builder.build(pats), repl)
    return f
