"""VectorMazeEnv — B independent maze env instances on one GPU, stepped by one HIP launch.

Wraps one libmazerl handle. All outputs live in persistent device tensors that every step /
reset overwrites in place (zero-copy for the learner); clone what you need to keep.

Observation parity with the reference (per instance):
  obs6[i]   = float32(concat(obs["agent"], obs["target"], obs["best dir"]))  as built by
              NeuralOffPolicyTrainer (lib/trainers/off_policy_trainer.py:156,169)
  window[i] = obs["window"] (3x15x15 f32, Enrich envs, lib/maze_handler.py:82-99)
  pos[i], best_dir[i] = obs["agent"], obs["best dir"] (plain envs)
  reward64[i] = the exact Python float the reference returns; reward[i] its float32 rounding.
The step tuple keeps the reference's order (obs, reward, truncated, terminated, info)
(gymnasium_env/envs/base_maze_env.py:210).
"""
import torch

from . import _native as N

ALGOS = {"r-prim": 0, "dfs": 1, "prim&kill": 2}


def _ptr(t):
    return None if t is None else t.data_ptr()


def bank_seed(env_seed):
    """The maze bank's Philox seed for an env seeded `env_seed` (0xBA4C0000 for the default env
    seed; distinct per shard because env seeds are 0x5EED0000 + the shard's first instance id)."""
    return (0xBA4C0000 + (int(env_seed) - 0x5EED0000) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF


class VectorMazeEnv:
    def __init__(self, num_envs, maze_dim, toroidal=False, enrich=True, device=None,
                 max_dim=None, algorithm="r-prim", seed=0x5EED0000, generate=True,
                 window=True, window_bits=True, reward64=False, pos=True, done_list=True,
                 host_scalars=False, candidates=1):
        if not torch.cuda.is_available():
            raise RuntimeError("VectorMazeEnv needs a HIP GPU (libmazerl.so has no CPU path)")
        self.lib = N.load()
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.num_envs = int(num_envs)
        self.maze_dim = int(maze_dim)
        self.max_dim = int(max_dim or maze_dim)
        self.toroidal, self.enrich = bool(toroidal), bool(enrich)
        cfg = N.Config(num_envs=self.num_envs, max_dim=self.max_dim, toroidal=int(toroidal),
                       enrich=int(enrich), device=self.device.index or 0)
        h = N.C.c_void_p()
        N.check(self.lib.mz_create(N.C.byref(cfg), N.C.byref(h)))
        self._h = h
        B, dev = self.num_envs, self.device
        kw = dict(device=dev)
        # host_scalars: the action and the per-instance scalars (reward, flags, position, best
        # dir) live in mapped page-locked host memory (mz_host_alloc) that the kernels read and
        # write directly — the single-env drop-ins' step() is then one launch + one stream sync
        # with no copies. They are CPU tensors then (valid until close(), which frees the
        # memory: clone what you keep); everything else stays in HBM.
        self._host = None
        self._dptr = {}
        if host_scalars:
            self._alloc_host(B, reward64, pos)
        else:
            self.reward = torch.zeros(B, dtype=torch.float32, **kw)
            self.reward64 = torch.zeros(B, dtype=torch.float64, **kw) if reward64 else None
            self.terminated = torch.zeros(B, dtype=torch.uint8, **kw)
            self.truncated = torch.zeros(B, dtype=torch.uint8, **kw)
            self.pos = torch.zeros(B, 2, dtype=torch.int32, **kw) if pos else None
            self.best_dir = torch.zeros(B, 2, dtype=torch.int32, **kw) if pos else None
            self.actions = torch.zeros(B, dtype=torch.int32, **kw)
        self.obs6 = torch.zeros(B, 6, dtype=torch.float32, **kw)
        self.window = torch.zeros(B, 3, 15, 15, dtype=torch.float32, **kw) if (enrich and window) else None
        self.window_bits = torch.zeros(B, 22, dtype=torch.int32, **kw) if (enrich and window_bits) else None
        self.done_idx = torch.zeros(B, dtype=torch.int32, **kw)
        self.done_count = torch.zeros(1, dtype=torch.int32, **kw)
        dp = self._dev_ptr
        self._out = N.StepOut(
            reward=dp(self.reward), reward64=dp(self.reward64), terminated=dp(self.terminated),
            truncated=dp(self.truncated), pos=dp(self.pos), best_dir=dp(self.best_dir),
            obs6=_ptr(self.obs6), window_bits=_ptr(self.window_bits), window=_ptr(self.window),
            done_idx=_ptr(self.done_idx) if done_list else None,
            done_count=_ptr(self.done_count) if done_list else None)
        self.seed = int(seed)
        self.epoch = 0
        self._bank = None
        self.algos_in_use = set()  # algorithm ids regeneration may ask for (sizes the bank)
        self._count_zero = True  # done_count is 0 (fresh, or consumed by reset_done)
        self._regen_dims = None
        if generate:
            self.generate(algorithm=algorithm, candidates=candidates)
            self.reset()

    # ---------------------------------------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _alloc_host(self, B, reward64, pos):
        import numpy as np
        fields = [("actions", np.int32, (B,)), ("reward", np.float32, (B,)),
                  ("reward64", np.float64, (B,)) if reward64 else None,
                  ("terminated", np.uint8, (B,)), ("truncated", np.uint8, (B,)),
                  ("pos", np.int32, (B, 2)) if pos else None,
                  ("best_dir", np.int32, (B, 2)) if pos else None]
        offs, total = [], 0
        for f in fields:
            if f is None:
                continue
            total = (total + 15) & ~15  # 16-B aligned fields
            offs.append((f, total))
            total += int(np.prod(f[2])) * np.dtype(f[1]).itemsize
        hp, dpp = N.C.c_void_p(), N.C.c_void_p()
        N.check(self.lib.mz_host_alloc(total, self.device.index or 0, N.C.byref(hp), N.C.byref(dpp)))
        self._host = hp
        raw = np.ctypeslib.as_array((N.C.c_uint8 * total).from_address(hp.value))
        for name in ("reward64", "pos", "best_dir"):
            setattr(self, name, None)
        for (name, dt, shape), off in offs:
            n = int(np.prod(shape)) * np.dtype(dt).itemsize
            t = torch.from_numpy(raw[off:off + n].view(dt).reshape(shape))
            setattr(self, name, t)
            self._dptr[t.data_ptr()] = dpp.value + off

    def _dev_ptr(self, t):
        """Device address of an output tensor (mapped host memory has its own)."""
        if t is None:
            return None
        return self._dptr.get(t.data_ptr(), t.data_ptr())

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mz_destroy(self._h)
            self._h = None
        if getattr(self, "_host", None) is not None:
            for name in ("actions", "reward", "reward64", "terminated", "truncated", "pos", "best_dir"):
                setattr(self, name, None)  # drop the views before the memory goes
            self.lib.mz_host_free(self._host)
            self._host = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------------------------------
    def generate(self, env_ids=None, algorithm="r-prim", dim=None, seed=None, rng="philox",
                 candidates=1):
        """New mazes for env_ids (None = all): gen_maze(shape, algorithm) per instance.
        rng="philox": Philox stream seed + env_id (every random choice uniform over the same
        candidates as the reference); rng="cpython": bit-exact — instance i gets the maze of
        `random.seed(seed + i); gen_maze((dim, dim), algorithm)` (MT19937 + CPython set order
        emulated on the GPU).
        candidates > 1 (Philox): the reference env's selection (BaseMazeEnv.generate_maze,
        base_maze_env.py:78-97; toroidal_maze_env.py:40-54) — the easiest of `candidates` mazes
        by McClendon difficulty, all on the GPU (mz_generate_best: candidate c of instance e is
        the maze of Philox seed + e * candidates + c, as best_of_mazes draws them)."""
        dim = int(dim or self.maze_dim)
        seed = self.seed if seed is None else int(seed)
        ids = None if env_ids is None else torch.as_tensor(env_ids, dtype=torch.int32, device=self.device)
        n = self.num_envs if ids is None else int(ids.numel())
        algo_t, algo_all = None, 0
        if isinstance(algorithm, str):
            algo_all = ALGOS[algorithm]
            self.algos_in_use.add(algo_all)
        elif isinstance(algorithm, int):
            algo_all = int(algorithm)
            self.algos_in_use.add(algo_all)
        else:
            algo_t = torch.as_tensor(algorithm, dtype=torch.uint8, device=self.device)
            if algo_t.numel() != n:
                raise ValueError("per-instance algorithm ids must match the env list")
            self.algos_in_use.update(ALGOS.values())
        mode = {"philox": N.MZ_RNG_PHILOX, "cpython": N.MZ_RNG_CPYTHON}[rng]
        if int(candidates) > 1:
            if mode != N.MZ_RNG_PHILOX:
                raise ValueError("best-of-C generation draws Philox candidates (rng='philox')")
            N.check(self.lib.mz_generate_best(self._h, _ptr(ids), n, _ptr(algo_t), algo_all, dim,
                                              seed & 0xFFFFFFFFFFFFFFFF, int(candidates),
                                              self._stream()))
            return self
        N.check(self.lib.mz_generate_ex(self._h, _ptr(ids), n, _ptr(algo_t), algo_all, dim,
                                        seed & 0xFFFFFFFFFFFFFFFF, mode, self._stream()))
        return self

    def select_stats(self, reset=False):
        """Best-of-C selection counters of this handle (bank refills + generate(candidates > 1)):
        {"unresolved": groups with a candidate neither the GPU kernels nor the host restatement
        scored (picked among the others), "near_ties": groups whose choice a 1-ulp log tie could
        change, "groups": selections made, "exact": groups the order-free screen could not decide
        (scored by the order-exact kernel), "host_scored": candidates that kernel declined, scored
        by the host restatement}."""
        out = torch.zeros(5, dtype=torch.int32, device=self.device)
        if hasattr(self.lib, "mz_select_stats_ex"):
            N.check(self.lib.mz_select_stats_ex(self._h, out.data_ptr(), 5, int(bool(reset)),
                                                self._stream()))
        else:  # an earlier round's library (MZ_LIB_OVERRIDE A/B runs): the first three
            N.check(self.lib.mz_select_stats(self._h, out.data_ptr(), int(bool(reset)),
                                             self._stream()))
        u, t, g, x, hs = (int(x) for x in out.cpu())
        return {"unresolved": u, "near_ties": t, "groups": g, "exact": x, "host_scored": hs}

    def set_debug(self, flags):
        """Test hooks of the best-of-C pipeline (mz_set_debug): 1 every group through the
        order-exact kernel, 2 even-numbered candidates host-scored, 4 identical candidates."""
        N.check(self.lib.mz_set_debug(self._h, int(flags)))

    def set_regen_dims(self, dims):
        """Per-instance size of a winner's next maze (uint8 device tensor [B], kept referenced
        here; 0 = the winner keeps its maze — update_maze past max_shape), or None: each
        instance's current size. Read by every later reset_done / reset_list(regen_won)."""
        if dims is None:
            self._regen_dims = None
            N.check(self.lib.mz_set_regen_dims(self._h, None))
            return
        t = torch.as_tensor(dims, device=self.device).to(torch.uint8).contiguous()
        if t.numel() != self.num_envs:
            raise ValueError("one size per instance")
        self._regen_dims = t
        N.check(self.lib.mz_set_regen_dims(self._h, t.data_ptr()))

    def generate_from_random(self, env_id=0, algorithm="r-prim", dim=None, rnd=None):
        """One maze for instance env_id drawn from a Python random.Random (default: the global
        `random` module) exactly as the reference's gen_maze((dim, dim), algorithm) would draw
        it (toroidal handles: gen_maze_no_border); the generator's state is advanced the same
        way (getstate -> GPU -> setstate)."""
        import random as _random
        import numpy as np
        rnd = _random if rnd is None else rnd
        dim = int(dim or self.maze_dim)
        algo = ALGOS[algorithm] if isinstance(algorithm, str) else int(algorithm)
        self.algos_in_use.add(algo)
        version, words, gauss = rnd.getstate()
        st = np.array(words, dtype=np.uint32)
        N.check(self.lib.mz_generate_state(self._h, int(env_id), dim, algo, st.ctypes.data,
                                           self._stream()))
        rnd.setstate((version, tuple(int(x) for x in st), gauss))
        return self

    def load_mazes(self, grids, start_goal, env_ids=None):
        """Import mazes bit-exactly (uint8 [n, dim, dim], int [n, 4] = sr, sc, gr, gc)."""
        import numpy as np
        g = np.ascontiguousarray(grids, dtype=np.uint8)
        sg = np.ascontiguousarray(start_goal, dtype=np.int32)
        ids = None if env_ids is None else np.ascontiguousarray(env_ids, dtype=np.int32)
        n, dim = g.shape[0], g.shape[1]
        N.check(self.lib.mz_load_mazes(self._h, g.ctypes.data, dim, sg.ctypes.data,
                                       None if ids is None else ids.ctypes.data, n,
                                       self._stream()))
        return self

    def set_algorithm(self, algorithm):
        if isinstance(algorithm, str):
            N.check(self.lib.mz_set_algorithm(self._h, None, ALGOS[algorithm], self._stream()))
            self.algos_in_use = {ALGOS[algorithm]}
        else:
            t = torch.as_tensor(algorithm, dtype=torch.uint8, device=self.device)
            N.check(self.lib.mz_set_algorithm(self._h, _ptr(t), 0, self._stream()))
            self.algos_in_use = set(ALGOS.values())

    # ---------------------------------------------------------------------------------------
    def _host_sync(self):
        """host_scalars: the scalar outputs are CPU tensors over mapped memory the kernels write
        asynchronously — wait for the launch before handing them back."""
        if self._host is not None:
            torch.cuda.current_stream(self.device).synchronize()

    def reset(self):
        N.check(self.lib.mz_reset_all(self._h, N.C.byref(self._out), self._stream()))
        self._host_sync()
        return self.obs(), {}

    def reset_list(self, idx, count=None, regen_won=False, seed=None):
        """Reset listed instances (device int32 list + optional device count)."""
        idx = torch.as_tensor(idx, dtype=torch.int32, device=self.device)
        if regen_won:
            self.epoch += 1
        N.check(self.lib.mz_reset_list(self._h, _ptr(idx), _ptr(count), int(idx.numel()),
                                       int(bool(regen_won)),
                                       (self.seed if seed is None else int(seed)) & 0xFFFFFFFFFFFFFFFF,
                                       self.epoch & 0xFFFFFFFF, N.C.byref(self._out),
                                       self._stream()))
        if count is not None and count.data_ptr() == self.done_count.data_ptr():
            self._count_zero = True  # the reset kernel consumed it
        self._host_sync()

    def reset_done(self, regen_won=False, seed=None):
        """Auto-reset every instance whose last step ended terminated|truncated (flag scan, no
        list); with regen_won the winners get a new maze first (win -> update_maze) — copied
        from the maze bank when one is enabled (enable_bank)."""
        if regen_won:
            self.epoch += 1
        N.check(self.lib.mz_reset_done(self._h, int(bool(regen_won)),
                                       (self.seed if seed is None else int(seed)) & 0xFFFFFFFFFFFFFFFF,
                                       self.epoch & 0xFFFFFFFF, N.C.byref(self._out),
                                       self._stream()))
        if regen_won and self._bank is not None:
            self._bank_tick()
        self._host_sync()

    # ---------------------------------------------------------------------------------------
    # Maze bank: winners' new mazes are generated ahead of time, in bulk, on a side stream.
    def enable_bank(self, slots=None, swap_every=8, algorithms=None, seed=None, dims=None,
                    candidates=1):
        """Two banks of `slots` mazes per algorithm (size maze_dim, or per size of `dims` — the
        variable-size envs): reset_done(regen_won=True) consumes the active one; every
        `swap_every` such calls the banks swap and the retired one is refilled on a side stream
        (ordered after the launches that consumed it; the main stream waits for a refill only
        when that bank comes back). Default slots: B / 8 (split over the sizes, >= 16 each).
        Default seed: derived from the env's seed, which carries the shard's first global
        instance id, so the ranks of a data-parallel run draw different replacement mazes.
        candidates > 1: every refilled slot is the easiest of `candidates` mazes by McClendon
        difficulty (the reference's generate_maze selection for a win's new maze,
        base_maze_env.py:78-97 via update_maze, off_policy_trainer.py:202), chosen on the GPU
        inside the refill (mz_bank_create_ex)."""
        if self._bank is not None:
            return
        if seed is None:
            seed = bank_seed(self.seed)
        dims = [self.maze_dim] if dims is None else sorted({int(d) for d in dims})
        K = int(slots or max(64 // len(dims) if len(dims) > 1 else 64,
                             self.num_envs // 8 // len(dims), 16))
        if algorithms is None:
            mask = sum(1 << i for i in self.algos_in_use) or 7
        else:
            ids = [ALGOS[a] if isinstance(a, str) else int(a) for a in algorithms]
            mask = sum(1 << i for i in set(ids))
        arr = (N.C.c_int32 * len(dims))(*dims)
        N.check(self.lib.mz_bank_create_ex(self._h, K, arr, len(dims), mask, int(candidates)))
        self._bank = dict(K=K, dims=dims, swap=int(swap_every), calls=0, cur=0, seed=int(seed),
                          side=torch.cuda.Stream(self.device), ready=[None, None],
                          candidates=int(candidates))
        st = self._stream()
        for b in (0, 1):
            N.check(self.lib.mz_bank_fill(self._h, b, self._bank["seed"], st))
        N.check(self.lib.mz_bank_use(self._h, 0))

    def _bank_tick(self):
        bk = self._bank
        bk["calls"] += 1
        if bk["calls"] % bk["swap"]:
            return
        old, new = bk["cur"], 1 - bk["cur"]
        main = torch.cuda.current_stream(self.device)
        if bk["ready"][new] is not None:
            main.wait_event(bk["ready"][new])
        N.check(self.lib.mz_bank_use(self._h, new))
        bk["cur"] = new
        consumed = torch.cuda.Event()
        consumed.record(main)
        side = bk["side"]
        side.wait_event(consumed)
        N.check(self.lib.mz_bank_fill(self._h, old, bk["seed"], side.cuda_stream))
        ev = torch.cuda.Event()
        ev.record(side)
        bk["ready"][old] = ev

    def bank_slot(self, bank, algorithm, dim, slot):
        """One bank slot's maze (synchronous; tests): (grid uint8 [N, N], (sr, sc, gr, gc))."""
        import numpy as np
        a = ALGOS[algorithm] if isinstance(algorithm, str) else int(algorithm)
        di = self._bank["dims"].index(int(dim))
        g = np.zeros((self.max_dim, self.max_dim), np.uint8)
        info = np.zeros(4, np.int32)
        N.check(self.lib.mz_bank_slot_grid(self._h, int(bank), a, di, int(slot), g.ctypes.data,
                                           info.ctypes.data))
        n = int(dim)
        return g.reshape(-1)[:n * n].reshape(n, n).copy(), tuple(int(x) for x in info)

    def bank_consumed(self, bank=None):
        """int32 [3] (a single-size bank) or [3, n_sizes]: slots of `bank` (default: the active
        one) consumed per algorithm id (and size)."""
        nd = len(self._bank["dims"])
        out = torch.zeros(3 * nd, dtype=torch.int32, device=self.device)
        b = self._bank["cur"] if bank is None else int(bank)
        N.check(self.lib.mz_bank_consumed(self._h, b, out.data_ptr(), self._stream()))
        return out if nd == 1 else out.view(3, nd)

    # ---------------------------------------------------------------------------------------
    # Checkpoint / resume (the reference has none for its envs)
    _OUTPUTS = ("reward", "reward64", "terminated", "truncated", "pos", "best_dir", "actions",
                "obs6", "window", "window_bits", "done_idx", "done_count")

    def state_dict(self):
        """Everything a resumed env needs to continue bit-exactly: the handle's device state
        (mz_state_save: mazes, tables, visit planes, per-instance state, the maze bank) as one
        uint8 device tensor, the last step's outputs (the next step's observation), and the
        host-side counters (regeneration epoch, bank rotation)."""
        main = torch.cuda.current_stream(self.device)
        if self._bank is not None:  # a refill still running on the side stream writes a bank
            for ev in self._bank["ready"]:
                if ev is not None:
                    main.wait_event(ev)
        n = N.C.c_uint64()
        N.check(self.lib.mz_state_bytes(self._h, N.C.byref(n)))
        blob = torch.empty(n.value, dtype=torch.uint8, device=self.device)
        N.check(self.lib.mz_state_save(self._h, blob.data_ptr(), n.value, self._stream()))
        out = {k: getattr(self, k).clone() for k in self._OUTPUTS if getattr(self, k) is not None}
        bank = None
        if self._bank is not None:
            bank = {k: self._bank[k] for k in ("K", "dims", "swap", "calls", "cur", "seed",
                                               "candidates")}
        return {"format": "mazerl.VectorMazeEnv/1", "num_envs": self.num_envs,
                "maze_dim": self.maze_dim, "max_dim": self.max_dim, "toroidal": self.toroidal,
                "enrich": self.enrich, "seed": self.seed, "epoch": self.epoch,
                "count_zero": self._count_zero, "algos_in_use": sorted(self.algos_in_use),
                "device_state": blob, "outputs": out, "bank": bank,
                "regen_dims": None if self._regen_dims is None else self._regen_dims.clone()}

    def load_state_dict(self, sd):
        """Restore a state_dict() into this env (same num_envs / max_dim / toroidal / enrich and,
        if the saved env had a maze bank, enable_bank() called with the same geometry first)."""
        if sd.get("format") != "mazerl.VectorMazeEnv/1":
            raise ValueError("not a VectorMazeEnv state_dict")
        bank = sd.get("bank")
        if (bank is None) != (self._bank is None) or (bank is not None and (
                bank["K"] != self._bank["K"] or list(bank["dims"]) != list(self._bank["dims"])
                or int(bank.get("candidates", 1)) != self._bank["candidates"])):
            raise ValueError("maze bank mismatch: call enable_bank() with the saved geometry "
                             "(or not at all) before load_state_dict()")
        blob = sd["device_state"].to(device=self.device, dtype=torch.uint8).contiguous()
        if self._bank is not None:  # a refill still running on the side stream would overwrite
            main = torch.cuda.current_stream(self.device)  # the loaded bank slots
            for ev in self._bank["ready"]:
                if ev is not None:
                    main.wait_event(ev)
        N.check(self.lib.mz_state_load(self._h, blob.data_ptr(), blob.numel(), self._stream()))
        for k, v in sd["outputs"].items():
            dst = getattr(self, k, None)
            if dst is None or tuple(dst.shape) != tuple(v.shape):
                raise ValueError(f"output {k!r}: this env's buffer does not match the saved one")
            dst.copy_(v)
        self.seed, self.epoch = int(sd["seed"]), int(sd["epoch"])
        self._count_zero = bool(sd["count_zero"])
        self.algos_in_use = set(sd.get("algos_in_use", ()))
        self.set_regen_dims(sd.get("regen_dims"))
        if bank is not None:
            self._bank.update(swap=int(bank["swap"]), calls=int(bank["calls"]),
                              cur=int(bank["cur"]), seed=int(bank["seed"]), ready=[None, None])
            # later refills run on the side stream: order them after this load
            self._bank["side"].wait_stream(torch.cuda.current_stream(self.device))
        self._host_sync()

    def reset_done_list(self, regen_won=False, seed=None):
        """Auto-reset from the step's device done list (consumes done_count)."""
        self.reset_list(self.done_idx, self.done_count, regen_won=regen_won, seed=seed)

    def step_host(self, action, env=0):
        """host_scalars envs: one instance's action straight into the mapped action slot, one
        launch, one stream synchronisation; the scalar outputs are then readable on the host."""
        if self._host is None:
            raise RuntimeError("step_host needs VectorMazeEnv(host_scalars=True)")
        self.actions[env] = int(action)
        N.check(self.lib.mz_step_ex(self._h, self._dev_ptr(self.actions), N.C.byref(self._out), 0,
                                    self._stream()))
        self._count_zero = False
        torch.cuda.current_stream(self.device).synchronize()

    def sync(self):
        torch.cuda.current_stream(self.device).synchronize()

    def step(self, actions, autoreset=False):
        """actions: int tensor [B] on the device (negative = observe only). With autoreset,
        instances whose previous step ended are reset by this launch instead (action ignored,
        reward 0, reset observation) — the trainer's env.reset() folded into the next step."""
        a = actions if (actions.dtype == torch.int32 and actions.device == self.device) else \
            actions.to(device=self.device, dtype=torch.int32)
        a = a.contiguous()
        flags = N.MZ_STEP_AUTORESET if autoreset else 0
        N.check(self.lib.mz_step_ex(self._h, self._dev_ptr(a), N.C.byref(self._out), flags,
                                    self._stream()))
        self._count_zero = False
        self._host_sync()
        return self.obs(), self.reward, self.truncated, self.terminated, {}

    def step_act(self, eps=1.0, greedy=None, seed=0, counter=0, actions_out=None, autoreset=False):
        """Fused epsilon-greedy act + step in one launch (actions taken -> actions_out; -1 for
        the instances an autoreset step resets)."""
        out = self.actions if actions_out is None else actions_out
        out_p = self._dev_ptr(out)
        eps_t = eps if torch.is_tensor(eps) else None
        g = None if greedy is None else greedy.to(dtype=torch.int64).contiguous()
        flags = N.MZ_STEP_COUNT_ZEROED if self._count_zero else 0
        if autoreset:
            flags |= N.MZ_STEP_AUTORESET
        N.check(self.lib.mz_step_act(self._h, _ptr(eps_t), float(eps) if eps_t is None else 0.0,
                                     _ptr(g), seed & 0xFFFFFFFFFFFFFFFF,
                                     counter & 0xFFFFFFFFFFFFFFFF, out_p,
                                     N.C.byref(self._out), flags, self._stream()))
        self._count_zero = False
        self._host_sync()
        return self.obs(), self.reward, self.truncated, self.terminated, {}

    def obs(self):
        o = {"obs6": self.obs6}
        if self.pos is not None:
            o["agent"], o["best dir"] = self.pos, self.best_dir
        if self.window is not None:
            o["window"] = self.window
        if self.window_bits is not None:
            o["window_bits"] = self.window_bits
        return o

    def direction_mask(self, probs=False, out=None):
        out = out if out is not None else torch.empty(self.num_envs, 4, dtype=torch.float32, device=self.device)
        N.check(self.lib.mz_direction_mask(self._h, int(bool(probs)), out.data_ptr(), self._stream()))
        return out

    def act(self, eps=1.0, greedy=None, seed=0, counter=0, out=None):
        """epsilon-greedy with the reference's masked exploration distribution."""
        out = out if out is not None else self.actions
        eps_t = eps if torch.is_tensor(eps) else None
        g = None if greedy is None else greedy.to(dtype=torch.int64).contiguous()
        N.check(self.lib.mz_act(self._h, _ptr(eps_t), float(eps) if eps_t is None else 0.0,
                                _ptr(g), seed & 0xFFFFFFFFFFFFFFFF, counter & 0xFFFFFFFFFFFFFFFF,
                                self._dev_ptr(out), self._stream()))
        if out is self.actions:
            self._host_sync()
        return out

    def expand_window(self, bits, out=None):
        n = bits.shape[0]
        out = out if out is not None else torch.empty(n, 3, 15, 15, dtype=torch.float32, device=bits.device)
        N.check(self.lib.mz_expand_window(bits.data_ptr(), out.data_ptr(), n, self._stream()))
        return out

    def meta(self, out=None):
        """int32 [B, 6]: N, start r, start c, goal r, goal c, max_steps (device tensor)."""
        out = out if out is not None else torch.empty(self.num_envs, 6, dtype=torch.int32, device=self.device)
        N.check(self.lib.mz_get_meta(self._h, out.data_ptr(), self._stream()))
        return out

    def maze_metrics(self, env_ids=None, out=None):
        """MetricsCalculator L, DE, D, AC, FDE, BDE of each listed instance's maze (euclidean),
        computed on the GPU: float64 [n, 6] device tensor (metrics_calculator.py)."""
        ids = None if env_ids is None else torch.as_tensor(env_ids, dtype=torch.int32, device=self.device)
        n = self.num_envs if ids is None else int(ids.numel())
        out = out if out is not None else torch.empty(n, 6, dtype=torch.float64, device=self.device)
        N.check(self.lib.mz_maze_metrics(self._h, _ptr(ids), n, out.data_ptr(), self._stream()))
        return out

    # ---------------------------------------------------------------------------------------
    def query(self, i):
        info = N.EnvInfo()
        N.check(self.lib.mz_query(self._h, int(i), N.C.byref(info)))
        return {k: getattr(info, k) for k, _ in N.EnvInfo._fields_}

    def grid(self, i):
        import numpy as np
        n = self.query(i)["n"]
        g = np.zeros((n, n), np.uint8)
        N.check(self.lib.mz_get_grid(self._h, int(i), g.ctypes.data))
        return g
