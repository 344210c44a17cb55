"""The draw rx_set_start_draws consumes (CPU, numpy only): MultiRacingEnv.reset's
np.random.shuffle(agent_order) on the 2-list [0, 1] (multi_racing_env.py:127-128)
takes exactly ONE MT19937 output u and swaps the cars when u & 1 == 0, and
np.random.randint(0, 2**32, dtype=np.uint32) returns those raw outputs one per
value -- so a device buffer of randint outputs drawn from a copy of the global
state replays the reference's start-slot sequence, and advancing the global
state by k randint draws equals k resets (rx/vector_env.py _NumpyStartDraws)."""
import numpy as np


def test_shuffle_of_two_is_one_raw_draw():
    for seed in (0, 1, 42, 2**31 - 1):
        np.random.seed(seed)
        orders = []
        for _ in range(500):
            order = [0, 1]
            np.random.shuffle(order)
            orders.append(order)
        s_shuffle = np.random.get_state()
        np.random.seed(seed)
        u = np.random.randint(0, 2**32, size=500, dtype=np.uint32)
        s_raw = np.random.get_state()
        assert [[0, 1] if v & 1 else [1, 0] for v in u] == orders
        assert s_shuffle[2] == s_raw[2] and np.array_equal(s_shuffle[1], s_raw[1])


def test_session_copy_then_advance_is_the_reference_stream():
    """begin(): outputs from a copy, global state restored; end(): advance by the
    number taken -- the global state then equals k shuffles, and the next draw
    (e.g. the PPO update's np.random.shuffle) is the reference's next draw."""
    np.random.seed(5)
    s0 = np.random.get_state()
    np.random.randint(0, 2**32, size=1000, dtype=np.uint32)
    np.random.set_state(s0)
    np.random.randint(0, 2**32, size=137, dtype=np.uint32)  # 137 resets taken
    nxt = np.random.permutation(64)
    np.random.seed(5)
    for _ in range(137):
        np.random.shuffle([0, 1])
    assert np.array_equal(np.random.permutation(64), nxt)
