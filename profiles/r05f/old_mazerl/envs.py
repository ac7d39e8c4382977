"""Single-env drop-ins for the reference's gym.Env classes (gymnasium_env/envs/*.py).

Each class keeps the reference's constructor, attributes and methods, including the swapped step
tuple (obs, reward, truncated, terminated, info) (base_maze_env.py:210), so the
reference's trainers/agents drive it unchanged. Underneath, every class is a 1-instance
VectorMazeEnv: generation, step, reset, masks and windows all run in libmazerl.so on the GPU.

  SimpleMazeEnv / SimpleEnrichMazeEnv                 simple_maze_env.py:14-158
  SimpleVariableMazeEnv / SimpleEnrichVariableMazeEnv simple_variable_maze_env.py:16-179
  ToroidalMazeEnv / ToroidalEnrichMazeEnv             toroidal_maze_env.py:15-172
  ToroidalVariableMazeEnv / ToroidalEnrichVariableMazeEnv  toroidal_variable_maze_env.py:15-194

Randomness: like the reference, mazes are drawn from Python's global `random`
state, and exactly as the reference draws them: the GPU generator runs gen_maze with CPython's
MT19937 stream and set iteration order (mz_generate_state), consuming the global stream draw for
draw, so `random.seed(s)` before construction gives the reference's own maze.
`reset(seed=...)` ignores the seed, as the reference does. The algorithm is the class-wide
BaseMazeEnv.ALGORITHM (set_algorithm changes it for every env, base_maze_env.py:60). New mazes
follow the reference's best-of-6 rule (base_maze_env.py:78-97): six candidates from the global
stream, the first with the smallest McClendon difficulty (native mz_difficulty) is kept.
"""
import random

import numpy as np
import torch

from .vector_env import ALGOS, VectorMazeEnv

try:  # optional: subclass gymnasium.Env when it is installed
    import gymnasium as _gym
    _EnvBase = _gym.Env
except Exception:  # pragma: no cover - gymnasium is not in this image
    _gym = None
    _EnvBase = object


class Discrete:
    def __init__(self, n):
        self.n = n

    def sample(self):
        return int(np.random.randint(self.n))


def _space_dict(shape, enrich):
    if _gym is not None:
        S = _gym.spaces
        d = {"agent": S.Box(low=np.array([0, 0]), high=np.array(shape), dtype=int),
             "target": S.Box(low=np.array([0, 0]), high=np.array(shape), dtype=int),
             "best dir": S.Box(-1, 1, shape=(2,), dtype=int)}
        if enrich:
            d["window"] = S.Box(-1, 1, shape=(3, 15, 15), dtype=float)
        return S.Dict(d)
    return {"agent": (2,), "target": (2,), "best dir": (2,), **({"window": (3, 15, 15)} if enrich else {})}


class BaseMazeEnv(_EnvBase):
    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": 4}
    ALGORITHM = "r-prim"
    ACTIONS = {0: np.array([1, 0]), 1: np.array([-1, 0]), 2: np.array([0, 1]), 3: np.array([0, -1])}
    TOROIDAL = False
    ENRICH = False
    VARIABLE = False
    START_SHAPE = None
    CANDIDATES = 6  # best-of-6 by difficulty, as the reference; set 1 for single-candidate

    def __init__(self, maze_shape, render_mode="human", device=None, _maze=None):
        self.render_mode = render_mode
        if self.VARIABLE:
            self.max_shape = tuple(maze_shape)
            shape = tuple(self.START_SHAPE)
            max_dim = max(self.max_shape[0], shape[0])
        else:
            shape = tuple(maze_shape)
            max_dim = shape[0]
        self.maze_shape = shape
        # host_scalars: action / reward / flags / position in mapped host memory, so step() is
        # one launch + one stream sync (no copies)
        self._venv = VectorMazeEnv(1, shape[0], toroidal=self.TOROIDAL, enrich=self.ENRICH,
                                   device=device, max_dim=max_dim, generate=False, reward64=True,
                                   host_scalars=True)
        self.action_space = Discrete(4)
        self.observation_space = _space_dict(shape, self.ENRICH)
        self.mazes = []
        self.next = 0
        self.cum_rew = 0
        if _maze is not None:
            self._load(*_maze)
        else:
            self._new_maze(shape[0])
        self._remember()
        self.reset()

    # --- construction helpers -----------------------------------------------------------------
    @classmethod
    def from_maze(cls, grid, start, goal, render_mode="human", device=None):
        """An env on a given maze (e.g. a reference-generated one), bypassing generation."""
        grid = np.asarray(grid, np.uint8)
        obj = cls.__new__(cls)
        shape = tuple(grid.shape)
        if cls.VARIABLE:
            BaseMazeEnv.__init__(obj, shape, render_mode, device, _maze=(grid, start, goal))
        else:
            BaseMazeEnv.__init__(obj, shape, render_mode, device, _maze=(grid, start, goal))
        return obj

    def _pull(self):
        q = self._venv.query(0)
        self._start_pos = (q["start_r"], q["start_c"])
        self._target_location = np.array([q["goal_r"], q["goal_c"]], dtype=np.int32)
        self.max_steps_taken = q["max_steps"]
        self.maze_map = self._venv.grid(0).astype(int).tolist()
        self.maze_shape = (q["n"], q["n"])

    def _difficulty_of_current(self):
        from .difficulty import maze_difficulty, toroidal_difficulty
        fn = toroidal_difficulty if self.TOROIDAL else maze_difficulty
        return fn(np.array(self.maze_map, np.uint8), self._start_pos,
                  tuple(int(x) for x in self._target_location))

    def _new_maze(self, n):
        """generate_maze (base_maze_env.py:78-97, toroidal_maze_env.py:40-54): CANDIDATES mazes
        generated on the GPU, the first with the smallest McClendon difficulty is kept."""
        best = None
        for _ in range(max(1, self.CANDIDATES)):
            # gen_maze / gen_maze_no_border from Python's global random, bit-exact
            self._venv.generate_from_random(0, ALGOS[BaseMazeEnv.ALGORITHM], dim=n)
            self._pull()
            if self.CANDIDATES <= 1:
                return
            d = self._difficulty_of_current()
            if best is None or d < best[0]:
                best = (d, np.array(self.maze_map, np.uint8), self._start_pos,
                        tuple(int(x) for x in self._target_location))
        self._load(best[1], best[2], best[3])

    def _load(self, grid, start, goal):
        grid = np.asarray(grid, np.uint8)
        self._venv.load_mazes(grid[None], np.array([[start[0], start[1], goal[0], goal[1]]]), env_ids=[0])
        self._pull()

    def _remember(self):
        if self.VARIABLE:
            self.mazes.append([self._start_pos, self.maze_shape, self.maze_map])
        else:
            self.mazes.append([self._start_pos, self.maze_map])

    # --- gym API -------------------------------------------------------------------------------
    def _obs(self):
        v = self._venv  # host-mapped outputs, written by the launch step()/reset() waited for
        pos = v.pos[0].numpy().astype(np.int32)
        bd = v.best_dir[0].numpy().astype(np.int64)
        self._agent_location = pos
        if self.ENRICH:
            shape = np.array(self.maze_shape)
            return {"agent": pos / shape, "target": self._target_location / shape, "best dir": bd,
                    "window": v.window[0].clone()}
        return {"agent": pos, "target": self._target_location, "best dir": bd}

    def _info(self):
        return {"distance": float(np.abs(self._agent_location - self._target_location).sum())}

    def reset(self, seed=None, options=None):
        self._venv.reset()
        self._venv.sync()
        obs = self._obs()
        self.cum_rew = 0
        return obs, self._info()

    def step(self, action):
        v = self._venv
        v.step_host(int(action))
        obs = self._obs()
        truncated = bool(v.truncated[0])
        terminated = bool(v.terminated[0])
        r = float(v.reward64[0])
        reward = -1 if truncated else (1 if terminated else r)  # the reference's int literals
        self.cum_rew += reward
        return obs, reward, truncated, terminated, self._info()

    def get_mask_direction(self, probs=False):
        m = self._venv.direction_mask(probs=bool(probs))[0].cpu().numpy()
        if probs and np.any(m == 0.25):
            return m.astype(np.float32)
        return m.astype(np.int32)

    # --- state views the reference exposes ----------------------------------------------------
    @property
    def env(self):  # agents reach the env as env.env (through a gymnasium wrapper)
        return self

    @property
    def steps_taken(self):
        return self._venv.query(0)["steps"]

    @property
    def consecutive_invalid_moves(self):
        return self._venv.query(0)["invalid_streak"]

    def set_algorithm(self, algorithm):
        if algorithm not in ALGOS:
            raise ValueError(algorithm)
        BaseMazeEnv.ALGORITHM = algorithm

    def get_algorithm(self):
        return BaseMazeEnv.ALGORITHM

    def get_maze_shape(self):
        return self.maze_shape

    def get_max_shape(self):
        return getattr(self, "max_shape", self.maze_shape)

    def get_maze_difficulty(self):
        # toroidal mazes are evaluated on the bordered maze (off_policy_trainer.py:194-196)
        return self._difficulty_of_current()

    def set_max_steps(self):
        self.max_steps_taken = self._venv.query(0)["max_steps"]

    # --- maze swaps (simple_maze_env.py:81-127, simple_variable_maze_env.py:93-147) -----------
    def update_maze(self):
        if self.VARIABLE:
            shape = tuple(a + b for a, b in zip(self.maze_shape, (4, 4)))
            if shape <= self.max_shape:
                self._new_maze(shape[0])
                self._remember()
                self.reset()
            else:
                random.shuffle(self.mazes)
            return
        self._new_maze(self.maze_shape[0])
        self._remember()
        self.reset()

    def update_visited_maze(self, remove=True):
        entry = self.mazes[self.next]
        if self.VARIABLE:
            start, shape, maze = entry
        else:
            start, maze = entry
        grid = np.array(maze, np.uint8)
        goal = tuple(int(x) for x in np.argwhere(grid == 2)[0])
        if remove:
            self.mazes.remove(entry)
        else:
            self.next += 1
        self._load(grid, start, goal)
        self.reset()

    def update_new_maze(self, shape=None):
        if shape is not None:
            n = shape[0]
        elif self.VARIABLE:
            n = random.sample([a for a in range(self.START_SHAPE[0], self.max_shape[0], 2)], 1)[0]
        else:
            n = self.maze_shape[0]
        self._new_maze(n)
        self.reset()

    # --- rendering (pygame view replaced by an RGB array; no display) -------------------------
    def render(self, mode="human", close=False):
        if close:
            return None
        colors = np.array([(46, 52, 64), (236, 239, 244), (163, 190, 140)], np.uint8)
        img = colors[np.array(self.maze_map, np.uint8)]
        r, c = self._agent_location
        img[r, c] = (94, 129, 172)
        return img

    def close(self):
        if getattr(self, "_venv", None) is not None:
            self._venv.close()
            self._venv = None


class SimpleMazeEnv(BaseMazeEnv):
    pass


class SimpleEnrichMazeEnv(SimpleMazeEnv):
    ENRICH = True
    WINDOW_DIM = 15


class SimpleVariableMazeEnv(BaseMazeEnv):
    VARIABLE = True
    START_SHAPE = (15, 15)


class SimpleEnrichVariableMazeEnv(SimpleVariableMazeEnv):
    ENRICH = True
    WINDOW_DIM = 15


class ToroidalMazeEnv(BaseMazeEnv):
    TOROIDAL = True


class ToroidalEnrichMazeEnv(ToroidalMazeEnv):
    ENRICH = True


class ToroidalVariableMazeEnv(BaseMazeEnv):
    TOROIDAL = True
    VARIABLE = True
    START_SHAPE = (29, 29)


class ToroidalEnrichVariableMazeEnv(ToroidalVariableMazeEnv):
    ENRICH = True


ENV_IDS = {  # gymnasium_env/__init__.py:3-31 (ids resolvable here, unlike the reference, Q17)
    "gymnasium_env/MazeEnv-v0": SimpleMazeEnv,
    "gymnasium_env/MazeEnv-v1": SimpleEnrichMazeEnv,
    "gymnasium_env/VariableMazeEnv-v0": SimpleVariableMazeEnv,
    "gymnasium_env/VariableMazeEnv-v1": SimpleEnrichVariableMazeEnv,
    "gymnasium_env/ToroidalMazeEnv-v0": ToroidalMazeEnv,
    "gymnasium_env/ToroidalMazeEnv-v1": ToroidalEnrichMazeEnv,
}


def make(env_id, *args, **kw):
    return ENV_IDS[env_id](*args, **kw)


def register_gymnasium():
    """Register the six ids with gymnasium when it is installed."""
    if _gym is None:
        return False
    for k, cls in ENV_IDS.items():
        _gym.register(id=k, entry_point=f"{__name__}:{cls.__name__}")
    return True
