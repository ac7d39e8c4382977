"""The single-env drop-in classes (mazerl.envs, the reference's 8 gym.Env names) replay the
reference's own traces with the reference's return types, and a NeuralOffPolicyTrainer-shaped
loop (lib/trainers/off_policy_trainer.py:144-263) runs against them with the drop-in DDQNAgent."""
import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import golden_io as G  # noqa: E402

pytestmark = pytest.mark.gpu

KIND_CLASS = {G.KIND_SIMPLE: "SimpleMazeEnv", G.KIND_ENRICH: "SimpleEnrichMazeEnv",
              G.KIND_TOR: "ToroidalMazeEnv", G.KIND_TOR_ENRICH: "ToroidalEnrichMazeEnv",
              G.KIND_VAR_ENRICH: "SimpleEnrichVariableMazeEnv"}


@pytest.fixture(scope="module")
def envs():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mazerl import envs as E
    return E


def test_dropin_replays_reference_traces(envs):
    for t in G.traces():
        cls = getattr(envs, KIND_CLASS[t["kind"]])
        env = cls.from_maze(t["grid"], t["start"], t["goal"])
        assert env.max_steps_taken == t["max_steps"]
        assert env.maze_map == t["grid"].astype(int).tolist()
        assert env._start_pos == t["start"] and tuple(env._target_location) == t["goal"]
        n = t["n"]
        for i, op in enumerate(t["op"][:400]):
            mi = env.get_mask_direction(probs=False)
            mp = env.get_mask_direction(probs=True)
            assert mi.dtype == np.int32
            np.testing.assert_array_equal(mi, t["mask_int"][i])
            np.testing.assert_array_equal(mp, t["mask_prob"][i])
            assert mp.dtype == (np.float32 if np.any(t["mask_prob"][i] == 0.25) else np.int32)
            if op == 4:
                obs, info = env.reset()
                r, tr, te = 0.0, False, False
            else:
                obs, r, tr, te, info = env.step(int(op))
            assert r == t["reward"][i] and tr == t["truncated"][i] and te == t["terminated"][i]
            if tr:
                assert isinstance(r, int) and r == -1
            np.testing.assert_array_equal(obs["best dir"], t["best_dir"][i])
            np.testing.assert_array_equal(obs["agent"], t["agent"][i])
            np.testing.assert_array_equal(obs["target"], t["target"][i])
            assert info["distance"] == t["distance"][i]
            if t["enrich"]:
                np.testing.assert_array_equal(obs["window"].cpu().numpy(), t["window"][i].astype(np.float32))
        env.close()


def test_reference_shaped_training_loop(envs):
    """The reference trainer's calling sequence against the drop-ins (train -> win -> update_maze,
    test(new=False) -> update_visited_maze, test(new=True) -> update_new_maze)."""
    from mazerl.agents.ddqn_agent import DDQNAgent
    random.seed(0)
    np.random.seed(0)
    env = envs.SimpleEnrichMazeEnv((15, 15))
    dev = torch.device("cuda")
    agent = DDQNAgent(env, learning_rate=1e-3, starting_epsilon=0.95, final_epsilon=0.1,
                      epsilon_decay=200, discount_factor=0.7, eta=1e-2, batch_size=16,
                      memory_size=2000, target_update_frequency=1, device=dev,
                      hidden_dim=64)
    wins = 0
    for episode in range(6):
        obs, _ = env.reset()
        state = (torch.tensor(np.concatenate([obs[k] for k in obs if k != "window"]), dtype=torch.float32,
                              device=dev).unsqueeze(0), obs["window"].to(dev).unsqueeze(0))
        done = False
        while not done:
            action = agent.get_action(state)
            nobs, reward, truncated, terminated, _ = env.env.step(action.item())
            nstate = (torch.tensor(np.concatenate([nobs[k] for k in nobs if k != "window"]),
                                   dtype=torch.float32, device=dev).unsqueeze(0),
                      nobs["window"].to(dev).unsqueeze(0))
            agent.memorize(state, action, reward, nstate)
            done = terminated or truncated
            state = nstate
            agent.optimize_model()
        if terminated:
            wins += 1
            env.env.update_maze()
        agent.update_hyperparameter(True)
        agent.scheduler_step()
        if agent.has_to_update(episode):
            agent.update_target()
    n_seen = len(env.mazes)
    assert n_seen == 1 + wins
    env.update_visited_maze(remove=True)
    assert len(env.mazes) == n_seen - 1
    env.set_algorithm("dfs")
    env.update_new_maze()
    assert env.get_algorithm() == "dfs" and envs.SimpleMazeEnv.ALGORITHM == "dfs"
    env.set_algorithm("r-prim")
    g = np.array(env.maze_map)
    assert g.shape == (15, 15) and (g == 2).sum() == 1
    env.close()


def test_q_agent_on_dropin_env_matches_reference(envs):
    """Config 1 plumbing: the tabular QAgent (str(obs) keys) on the GPU drop-in SimpleMazeEnv
    yields the reference's keys and Q-table for the same op sequence (agents/q_agent.py:56-67)."""
    from mazerl.agents.q_agent import QAgent
    fx = G.load("agents.npz")
    t = [t for t in G.traces() if t["kind"] == G.KIND_SIMPLE][int(fx["q.trace_index"])]
    env = envs.SimpleMazeEnv.from_maze(t["grid"], t["start"], t["goal"])
    ag = QAgent(env, learning_rate=0.1, initial_epsilon=0.95, epsilon_decay=40,
                final_epsilon=0.05, discount_factor=0.7, eta=0.01)
    obs, _ = env.reset()
    keys = []
    for op in t["op"][:600]:
        if op == 4:
            obs, _ = env.reset()
            continue
        nobs, r, tr, te, _ = env.step(int(op))
        ag.update(obs, int(op), r, te, nobs)
        keys.append(str(obs))
        obs = nobs
    assert keys == list(fx["q.obs"])
    assert sorted(ag.q_values) == list(fx["q.keys"])
    for k, v in zip(fx["q.keys"], fx["q.values"]):
        np.testing.assert_array_equal(ag.q_values[str(k)], v)
    env.close()


def test_best_of_6_generation(envs):
    """generate_maze keeps the first of 6 candidates with the smallest difficulty
    (base_maze_env.py:78-97); the candidates come from the global `random` stream exactly as
    gen_maze draws them (checked against the oracle's CPython restatement)."""
    import pyoracle as O
    from mazerl.difficulty import maze_difficulty
    envs.BaseMazeEnv.ALGORITHM = "r-prim"
    random.seed(77)
    env = envs.SimpleMazeEnv((21, 21))
    st = O.mt_state(77)
    cands = []
    for _ in range(6):
        s, g, grid = O.generate_py(21, 0, st)
        cands.append((maze_difficulty(grid, s, g), grid))
    best = min(range(6), key=lambda i: (cands[i][0], i))
    assert np.array_equal(np.array(env.maze_map), cands[best][1])
    assert env.get_maze_difficulty() == cands[best][0]
    env.close()


def test_variable_env_growth(envs):
    random.seed(1)
    env = envs.SimpleVariableMazeEnv((23, 23))
    assert env.get_maze_shape() == (15, 15) and env.get_max_shape() == (23, 23)
    env.update_maze()
    assert env.get_maze_shape() == (19, 19)
    env.update_maze()
    assert env.get_maze_shape() == (23, 23)
    env.update_maze()  # > max_shape: shuffles the learned mazes instead (:111-112)
    assert env.get_maze_shape() == (23, 23) and len(env.mazes) == 3
    env.update_new_maze()
    assert env.get_maze_shape()[0] in (15, 17, 19, 21)
    obs, _ = env.reset()
    assert set(obs) == {"agent", "target", "best dir"}
    env.close()
    tv = envs.ToroidalEnrichVariableMazeEnv((41, 41))
    assert tv.get_maze_shape() == (29, 29)
    obs, _ = tv.reset()
    assert obs["window"].shape == (3, 15, 15)
    tv.close()


ENV_CLASS = {"simple": "SimpleMazeEnv", "simple_enrich": "SimpleEnrichMazeEnv",
             "toroidal": "ToroidalMazeEnv", "toroidal_enrich": "ToroidalEnrichMazeEnv",
             "simple_variable": "SimpleVariableMazeEnv",
             "toroidal_variable": "ToroidalVariableMazeEnv"}


def test_dropin_constructor_matches_reference_after_seed(envs):
    """random.seed(s); Env(shape) builds the reference's own maze (tests/golden/envs.npz: the
    reference's constructors, best-of-6 from the global stream) and leaves Python's global
    random stream exactly where the reference leaves it."""
    ALG = ["r-prim", "dfs", "prim&kill"]
    saved = envs.BaseMazeEnv.ALGORITHM
    try:
        for e in G.envs():
            envs.BaseMazeEnv.ALGORITHM = ALG[e["algo"]]
            random.seed(e["seed"])
            env = getattr(envs, ENV_CLASS[e["kind"]])((e["ctor"], e["ctor"]))
            probe = random.getrandbits(32)
            key = (e["kind"], e["ctor"], e["algo"], e["seed"])
            assert env.maze_map == e["grid"].astype(int).tolist(), key
            assert env._start_pos == e["start"] and tuple(env._target_location) == e["goal"], key
            assert env.max_steps_taken == e["max_steps"], key
            assert probe == e["probe"], key
            env.close()
    finally:
        envs.BaseMazeEnv.ALGORITHM = saved


def test_gen_maze_functions_match_reference_mazes(envs):
    """mazerl.lib.maze_generation.gen_maze / gen_maze_no_border (maze_generation.py:6-56) after
    random.seed(s): the reference's own mazes (the 240 golden ones: 3 algorithms x 5 sizes x 8
    seeds), start / goal, gen_maze_no_border's difficulty on the bordered maze, and the global
    random stream left where the reference leaves it (checked against the oracle's CPython
    restatement). Even sizes raise IndexError (Q4)."""
    import random
    import pyoracle as O
    from mazerl.lib.maze_generation import gen_maze, gen_maze_no_border
    for name, fn, tor in (("gen_euclid.npz", gen_maze, False), ("gen_toroid.npz", gen_maze_no_border, True)):
        for m in G.mazes(name):
            algo = G.ALGOS[m["algo"]]
            random.seed(m["seed"])
            out = fn((m["n"], m["n"]), algo)
            key = (name, algo, m["n"], m["seed"])
            np.testing.assert_array_equal(np.array(out[2]), m["grid"], err_msg=str(key))
            assert out[0] == m["start"] and out[1] == m["goal"], key
            if tor and not np.isnan(m["difficulty"]):
                assert out[3] == pytest.approx(m["difficulty"], rel=1e-15, abs=0), key
            if not tor and m["n"] <= 41:
                st = O.mt_state(m["seed"])
                O.generate_py(m["n"], m["algo"], st)
                assert list(st) == list(random.getstate()[1]), key
    with pytest.raises(IndexError):
        gen_maze((40, 40), "r-prim")
