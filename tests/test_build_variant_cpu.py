"""Build-variant safety: the loader refuses (or rebuilds) a library whose
stamp records extra compile macros or a non-default optimisation level, unless
PMD_ALLOW_VARIANT=1 -- e.g. the timing-only -DPMD_TIMING_NO_ATOMICS build, which zeroes every
BN statistic, can never bench silently; bench.py records the library digest and flags."""
import pytest

from pytorch_multiprocessing_distributed_amd.ops import native


class _FakeBuild:
    def __init__(self, stamp, tmp_path):
        self.stamp = stamp
        self.lib = tmp_path / "_C.so"
        self.lib.write_bytes(b"\0")
        self.built = []

    def read_stamp(self):
        return self.stamp

    def target_path(self):
        return str(self.lib)

    def source_digest(self):
        return "src"

    def build(self, verbose=True, force=False):
        self.built.append(force)


def _stamp(**kw):
    st = {"sources": "src", "library": "ab" * 32, "arch": "gfx950", "opt": ["-O3"], "extra_cflags": ""}
    st.update(kw)
    return st


@pytest.fixture
def env(monkeypatch):
    for k in ("PMD_ALLOW_VARIANT", "PMD_EXTRA_CFLAGS", "PMD_NO_AUTOBUILD", "PMD_EXT_DIR"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_production_stamp_loads(env, tmp_path):
    fb = _FakeBuild(_stamp(), tmp_path)
    env.setattr(native, "_build_module", lambda: fb)
    native._ensure_built()
    assert fb.built == []
    assert native.variant_reason(fb.stamp) == ""


@pytest.mark.parametrize("variant", [{"extra_cflags": "-DPMD_TIMING_NO_ATOMICS=1"}, {"opt": ["-O1", "-g"]}])
def test_variant_stamp_is_refused_or_rebuilt(env, tmp_path, variant):
    fb = _FakeBuild(_stamp(**variant), tmp_path)
    env.setattr(native, "_build_module", lambda: fb)
    env.setenv("PMD_NO_AUTOBUILD", "1")
    with pytest.raises(ImportError, match="variant library"):
        native._ensure_built()
    env.delenv("PMD_NO_AUTOBUILD")
    native._ensure_built()                 # rebuilt with the production flags, forced
    assert fb.built == [True]
    env.setenv("PMD_ALLOW_VARIANT", "1")   # explicitly wanted (A/B scripts): loads as is
    fb.built.clear()
    native._ensure_built()
    assert fb.built == []


def test_extra_cflags_env_needs_allow_variant(env, tmp_path):
    fb = _FakeBuild(_stamp(), tmp_path)
    env.setattr(native, "_build_module", lambda: fb)
    env.setenv("PMD_EXTRA_CFLAGS", "-DPMD_TIMING_NO_ATOMICS=3")
    with pytest.raises(ImportError, match="PMD_ALLOW_VARIANT"):
        native._ensure_built()


def test_stamp_info_reports_digest_and_flags(env, tmp_path):
    fb = _FakeBuild(_stamp(extra_cflags="-DX=1"), tmp_path)
    env.setattr(native, "_build_module", lambda: fb)
    info = native.stamp_info()
    assert info["lib_digest"] == ("ab" * 32)[:16] and info["extra_cflags"] == "-DX=1"
    assert info["opt"] == "-O3"
