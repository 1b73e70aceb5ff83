"""The C-ABI boundary (include/factorysim.h) without a GPU: the HIP library loads, exports every function
the header declares, the Python binding registers the same set, and the product path refuses to run
without a device instead of falling back to the CPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "factorysim.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fm_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from factory_marl_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfactorysim.so not built (run `python __graft_entry__.py`)")
    return _lib.load()


def test_header_declares_the_entry_points():
    fns = header_functions()
    for need in ["fm_create", "fm_destroy", "fm_reset", "fm_step", "fm_get_state", "fm_set_state", "fm_set_stream"]:
        assert need in fns


def test_library_exports_every_header_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_binding_registers_the_header_set():
    from factory_marl_amd import _lib

    assert sorted(_lib.EXPORTED) == header_functions()


def test_abi_version_and_config_size(lib):
    """the library's ABI version and fm_config size are the header's (the binding checks both at load)"""
    from factory_marl_amd import _lib

    m = re.search(r"#define FM_ABI_VERSION (\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.ABI_VERSION == lib.fm_abi_version()
    assert lib.fm_config_size() == C.sizeof(_lib.FmConfig)


def test_config_defaults_match_the_reference(lib):
    from factory_marl_amd import _lib

    c = _lib.FmConfig()
    lib.fm_config_default(C.byref(c))
    # challenge_env/base_env.py defaults
    assert c.num_arms == 2 and c.max_num_objects == 10
    assert c.initial_conveyor_speed == pytest.approx(0.1)
    assert c.conveyor_acceleration == pytest.approx(0.001)
    assert c.pt_time == pytest.approx(0.2)
    assert c.force_contact_threshold == pytest.approx(200.0)
    assert c.control_frequency == pytest.approx(10.0)
    assert c.spawn_freq_increase == pytest.approx(1.001)


def test_create_fails_loudly_without_a_device(lib):
    """no GPU here: fm_create must return an error (never a CPU fallback)"""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from factory_marl_amd import _lib

    c = _lib.FmConfig()
    lib.fm_config_default(C.byref(c))
    c.num_arenas = 2
    c.max_num_objects = 4
    h = C.c_void_p()
    rc = lib.fm_create(C.byref(c), 0, None, C.byref(h))
    assert rc != 0
    assert lib.fm_last_error().decode()


def test_vec_env_raises_without_library(monkeypatch, tmp_path):
    from factory_marl_amd import _lib

    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "EXP_LIB_PATH", str(tmp_path / "missing_exp.so"))
    monkeypatch.setattr(_lib, "_LIBS", {})
    with pytest.raises(_lib.FactorySimError):
        _lib.load()
    with pytest.raises(_lib.FactorySimError):
        _lib.load(experimental=True)


def test_state_record_roundtrip():
    from factory_marl_amd import state as st

    A, K = 2, 4
    nq, nv, nu, nd, ni = st.sizes(A, K)
    rng = np.random.default_rng(0)
    d = rng.normal(size=nd)
    i = rng.integers(-5, 100, ni).astype(np.int32)
    r = rng.integers(0, 2**63, 4, dtype=np.uint64)
    rec = st.pack(A, K, d, i, r)
    assert rec.nbytes == st.record_bytes(A, K)
    d2, i2, r2 = st.unpack(A, K, rec)
    assert np.array_equal(d, d2) and np.array_equal(i, i2) and np.array_equal(r, r2)
    f = st.fields(A, K, d)
    assert f["qpos"].shape == (nq,) and f["ctrl_target"].shape == (nu,) and f["episode_return"].shape == (1,)
    # sizes of the benchmark scene (nq 47, nv 43, nu 17, obs 100)
    assert (nq, nv, nu) == (47, 43, 17)


def test_config1_steps_on_the_cpu_backend_and_matches_the_oracle(lib, oracle):
    """BASELINE config 1 (one env, 2 arms x 4 objects, random policy -- the reference's visualisation.py:32-77 loop)
    through the same C ABI on device = -1 (the kernel's own sources on the host, fm_cpu.cpp): started from the
    oracle's reset record, 30 free-running env-steps against the oracle's; fp64, state within 1e-6 relative,
    task integers / RNG / flags bit for bit"""
    import torch

    from factory_marl_amd import FactoryVecEnv, state as st
    from factory_marl_amd.environments import run_kwargs

    A, K = 2, 4
    e = oracle.Env(A, K, 42, weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    kw = run_kwargs("AllFullRLProgressRewardEnv", num_arms=A, max_num_objects=K, seed=42)
    kw["small_action_norm_reward_factor"] = 0.1
    env = FactoryVecEnv(1, env_kwargs=kw, device=-1, precision="fp64")
    env.reset()
    env.set_state(st.pack(A, K, *e.export_state())[None])
    rng = np.random.default_rng(1)
    for t in range(30):
        a = rng.uniform(-1, 1, 8 * A).astype(np.float32)
        obs, rew, term, _, _ = e.step(a)
        g_obs, g_rew, g_term, _ = env.step_tensors(torch.as_tensor(a[None]))
        assert bool(g_term[0]) == term, t
        assert float(g_rew[0]) == pytest.approx(rew, abs=1e-6), t
        assert np.abs(g_obs[0].numpy() - obs).max() <= 1e-5, t
        gd, gi, gr = st.unpack(A, K, env.get_state()[0])
        d, i, r = e.export_state()
        assert np.array_equal(gi, i) and np.array_equal(gr, r), t
        qd, vd = __import__("parity_util").state_err(A, K, gd, d)
        assert max(qd.max(), vd.max()) <= 1e-6, (t, qd.max(), vd.max())
        if term:
            break
    env.close()
