"""Stream handling of the C ABI (fm_set_stream / fm_destroy) on the GPU.

* fm_destroy destroys only the private stream fm_create made, never a stream the caller handed in.
* Changing streams orders the new stream after the work queued on the old one: stepping on two
  alternating non-blocking torch streams gives the same arena state, bit for bit, as stepping on one.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]


def _env(n=64):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42), precision="fp32")
    env.reset()
    return env


def _actions(n, steps, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    return [torch.rand(n, 16, device=dev, generator=g) * 2 - 1 for _ in range(steps)]


def test_destroy_leaves_caller_stream_usable():
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        env = _env(8)
        env.step_tensors(_actions(8, 1, env.device)[0])
        env.close()  # must not destroy s
        x = torch.ones(1024, device="cuda") * 2
    s.synchronize()
    ev = torch.cuda.Event()
    ev.record(s)
    ev.synchronize()
    assert float(x.sum().item()) == 2048.0


def test_alternating_streams_match_single_stream():
    n, steps = 256, 6
    ref = _env(n)
    acts = _actions(n, steps, ref.device)
    for a in acts:
        ref.step_tensors(a)
    ref.sync()
    want = ref.get_state()
    ref.close()

    env = _env(n)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for i, a in enumerate(acts):
        s = s1 if i % 2 == 0 else s2
        s.wait_stream(torch.cuda.current_stream())  # the actions were made on the default stream
        with torch.cuda.stream(s):
            env.step_tensors(a)
    with torch.cuda.stream(s2):
        got = env.get_state()
    env.close()
    assert np.array_equal(got, want)


def test_longest_first_dispatch_does_not_change_results(monkeypatch):
    """the env-step's workgroup -> arena map is re-sorted every step by the arenas' last durations
    (lpt_order_kernel); stepping with it and with the plain blockIdx order
    (FACTORYSIM_NO_LPT, read at fm_create) gives the same observations and arena state bit for bit"""
    n, steps = 512, 40
    lpt = _env(n)
    monkeypatch.setenv("FACTORYSIM_NO_LPT", "1")
    plain = _env(n)
    monkeypatch.delenv("FACTORYSIM_NO_LPT")
    for a in _actions(n, steps, lpt.device):
        lpt.step_tensors(a)
        plain.step_tensors(a)
    lpt.sync()
    plain.sync()
    assert torch.equal(lpt.obs, plain.obs)
    assert np.array_equal(lpt.get_state(), plain.get_state())
    # the durations the order is sorted by (fm_get_costs): every arena stepped, each env-step under a second
    c = lpt.costs()
    assert c.shape == (n,) and (c > 0).all() and (c < 100_000_000).all()  # 100 MHz wall clock ticks
    from factory_marl_amd._lib import FactorySimError

    with pytest.raises(FactorySimError):
        plain.costs()  # FACTORYSIM_NO_LPT: no per-arena costs kept
    lpt.close()
    plain.close()
