"""Offline stand-ins for `gymnasium` and `pygame` so the reference's *library* code imports here.

Fixture-generation infrastructure only (never imported by the product or on the GPU box).
The reference pins gymnasium 1.0.0 / pygame 2.6.1 (README.md:6-13); neither is installed in this
image. The reference env only needs: `gym.Env`, `spaces.{Discrete,Box,Dict}`,
`envs.registration.register` and (scripts only) `wrappers`; the view only needs pygame calls that
draw. Rendering has no effect on any value the env returns, so no-op drawing is
faithful for every quantity recorded in the fixtures.
"""
import sys
import types

import numpy as np


def install():
    if "gymnasium" in sys.modules and getattr(sys.modules["gymnasium"], "_MAZERL_STUB", False):
        return
    # ---- gymnasium ----
    gym = types.ModuleType("gymnasium")
    gym._MAZERL_STUB = True

    class Env:
        metadata = {}

        def close(self):
            pass

    class Discrete:
        def __init__(self, n, *a, **k):
            self.n = int(n)

        def sample(self):
            return int(np.random.randint(self.n))

    class Box:
        def __init__(self, low=None, high=None, shape=None, dtype=None, *a, **k):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class Dict:
        def __init__(self, spaces=None, *a, **k):
            self.spaces = spaces

    spaces = types.ModuleType("gymnasium.spaces")
    spaces.Discrete, spaces.Box, spaces.Dict = Discrete, Box, Dict
    envs = types.ModuleType("gymnasium.envs")
    registration = types.ModuleType("gymnasium.envs.registration")
    registration.register = lambda *a, **k: None
    envs.registration = registration
    wrappers = types.ModuleType("gymnasium.wrappers")

    class RecordEpisodeStatistics:
        def __init__(self, env, *a, **k):
            self.env = env
            self.action_space = env.action_space

        def reset(self, *a, **k):
            return self.env.reset(*a, **k)

        def step(self, a):
            return self.env.step(a)

        def close(self):
            pass

        def __getattr__(self, name):
            return getattr(self.env, name)

    wrappers.RecordEpisodeStatistics = RecordEpisodeStatistics
    gym.Env, gym.spaces, gym.envs, gym.wrappers = Env, spaces, envs, wrappers
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces, "gymnasium.envs": envs,
                        "gymnasium.envs.registration": registration,
                        "gymnasium.wrappers": wrappers})

    # ---- pygame (explicit attributes only; no catch-all __getattr__, torch's inspect breaks) ----
    pg = types.ModuleType("pygame")

    class _Surface:
        def __init__(self, *a, **k):
            pass

        def convert(self):
            return self

        def convert_alpha(self):
            return self

        def blit(self, *a, **k):
            pass

    class _Rect:
        def __init__(self, *a, **k):
            pass

    display = types.ModuleType("pygame.display")
    display.set_caption = lambda *a, **k: None
    display.init = lambda *a, **k: None
    display.quit = lambda *a, **k: None
    display.set_mode = lambda *a, **k: _Surface()
    display.flip = lambda *a, **k: None
    display.update = lambda *a, **k: None
    display.get_surface = lambda *a, **k: _Surface()
    draw = types.ModuleType("pygame.draw")
    draw.rect = lambda *a, **k: None
    event = types.ModuleType("pygame.event")
    event.get = lambda *a, **k: []
    surfarray = types.ModuleType("pygame.surfarray")
    surfarray.array3d = lambda *a, **k: np.zeros((1, 1, 3))
    pg.init = lambda *a, **k: None
    pg.quit = lambda *a, **k: None
    pg.Surface, pg.Rect, pg.QUIT = _Surface, _Rect, 256
    pg.display, pg.draw, pg.event, pg.surfarray = display, draw, event, surfarray
    sys.modules.update({"pygame": pg, "pygame.display": display, "pygame.draw": draw,
                        "pygame.event": event, "pygame.surfarray": surfarray})
