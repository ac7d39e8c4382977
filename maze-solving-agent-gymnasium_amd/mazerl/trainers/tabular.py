"""Config 1 (BASELINE configs[0]): the reference's tabular loop, OffPolicyTrainer
(lib/trainers/off_policy_trainer.py:11-133), over the drop-in envs (mazerl.envs: one instance on
the GPU handle each) and agents (mazerl.agents.q_agent.QAgent).

train(n_episodes) (:21-86): one episode per iteration — get_action / step / update until
terminated or truncated, a win -> env.update_maze() (the new maze appended to env.mazes; the
variable-size envs stop at their max shape), then update_hyperparameter(cumulative reward grew).
The reference logs each win's McClendon difficulty; that is logging only and left out.
test(num_mazes, new) (:88-123): new -> update_new_maze(), else update_visited_maze(remove=True) —
the seen-maze replay over env.mazes; one greedy-or-epsilon episode each (get_action as in
training). Returns win counts and env steps (the reference logs them)."""
import time


class TabularTrainer:
    def __init__(self, env, agent):
        self.env, self.agent = env, agent
        base = getattr(env, "env", env)
        self.is_maze_variable = hasattr(base, "get_max_shape") and \
            type(base).__name__.endswith("VariableMazeEnv")
        self.env_steps = 0
        self.wins = 0

    def _base(self):
        return getattr(self.env, "env", self.env)

    def train(self, n_episodes):
        """Returns (wins, env steps, seconds)."""
        t0 = time.perf_counter()
        wins = steps = 0
        prev_cum = 0.0
        for _ in range(n_episodes):
            obs, _ = self.env.reset()
            done, win, cumulative = False, False, 0.0
            while not done:
                action = self.agent.get_action(obs)
                nxt, reward, truncated, terminated, _ = self.env.step(action)  # (Q1: swapped)
                cumulative += reward
                self.agent.update(obs, action, reward, terminated, nxt)
                done = terminated or truncated
                win = terminated
                obs = nxt
                steps += 1
            if win:
                wins += 1
                self._base().update_maze()
                if self.is_maze_variable and \
                        self._base().get_maze_shape() >= self._base().get_max_shape():
                    break
            self.agent.update_hyperparameter(cumulative > prev_cum)
            prev_cum = cumulative
        self.env_steps += steps
        self.wins += wins
        return wins, steps, time.perf_counter() - t0

    def test(self, num_mazes, new):
        """Win rate over num_mazes episodes (new mazes, or the visited ones popped in order)."""
        win = 0
        for _ in range(num_mazes):
            if new:
                self._base().update_new_maze()
            else:
                self._base().update_visited_maze(remove=True)
            obs, _ = self.env.reset()
            done = False
            while not done:
                action = self.agent.get_action(obs)
                obs, _, truncated, terminated, _ = self.env.step(action)
                if terminated:
                    win += 1
                    done = True
                else:
                    done = truncated
        return win / max(1, num_mazes)
