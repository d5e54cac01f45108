"""Play-time state / reward logger (legged_gym/utils/logger.py:36-136): per-step scalar states of one
robot, per-episode reward sums, a 3 x 3 figure of the logged states and the average reward per
term.  The reference plots in a child process with plt.show(); headless here, the figure is
rendered with matplotlib's Agg backend into a PNG (`plot_states(path)`), in the calling process
(no window, no extra process to join)."""
from collections import defaultdict

import numpy as np

# (row, col) of each panel: (x-key or None = time, [(series key, label)], xlabel, ylabel, title)
_PANELS = {
    (0, 0): (None, [("base_vel_x", "measured"), ("command_x", "commanded")], "time [s]", "base lin vel [m/s]",
             "Base velocity x"),
    (0, 1): (None, [("base_vel_y", "measured"), ("command_y", "commanded")], "time [s]", "base lin vel [m/s]",
             "Base velocity y"),
    (0, 2): (None, [("base_vel_yaw", "measured"), ("command_yaw", "commanded")], "time [s]", "base ang vel [rad/s]",
             "Base velocity yaw"),
    (1, 0): (None, [("dof_pos", "measured"), ("dof_pos_target", "target")], "time [s]", "Position [rad]",
             "DOF Position"),
    (1, 1): (None, [("dof_vel", "measured"), ("dof_vel_target", "target")], "time [s]", "Velocity [rad/s]",
             "Joint Velocity"),
    (1, 2): (None, [("base_vel_z", "measured")], "time [s]", "base lin vel [m/s]", "Base velocity z"),
    (2, 0): (None, [("contact_forces_z", "force")], "time [s]", "Forces z [N]", "Vertical Contact forces"),
    (2, 1): ("dof_vel", [("dof_torque", "measured")], "Joint vel [rad/s]", "Joint Torque [Nm]",
             "Torque/velocity curves"),
    (2, 2): (None, [("dof_torque", "measured")], "time [s]", "Joint Torque [Nm]", "Torque"),
}


class Logger:
    def __init__(self, dt):
        self.state_log = defaultdict(list)
        self.rew_log = defaultdict(list)
        self.dt = dt
        self.num_episodes = 0

    def log_state(self, key, value):
        self.state_log[key].append(value)

    def log_states(self, states):
        for key, value in states.items():
            self.log_state(key, value)

    def log_rewards(self, episode_infos, num_episodes):
        """episode_infos: extras["episode"] (per-term means over the envs reset this step, as
        scalar tensors); the sums are weighted by the number of episodes (logger.py:51-55)."""
        for key, value in episode_infos.items():
            if "rew" in key:
                self.rew_log[key].append(float(value) * num_episodes)
        self.num_episodes += num_episodes

    def reset(self):
        self.state_log.clear()
        self.rew_log.clear()

    def average_rewards(self):
        """{term: average reward per second over the logged episodes} (what print_rewards prints)."""
        return {k: float(np.sum(v)) / self.num_episodes for k, v in self.rew_log.items()} if self.num_episodes else {}

    def print_rewards(self):
        print("Average rewards per second:")
        for key, mean in self.average_rewards().items():
            print(f" - {key}: {mean}")
        print(f"Total number of episodes: {self.num_episodes}")

    def plot_states(self, path="states.png"):
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        log = self.state_log
        n = max((len(v) for v in log.values()), default=0)
        time = np.linspace(0, n * self.dt, n)
        fig, axs = plt.subplots(3, 3, figsize=(15, 10))
        for (r, c), (xkey, series, xl, yl, title) in _PANELS.items():
            a = axs[r, c]
            for key, label in series:
                y = log.get(key)
                if not y:
                    continue
                x = time if xkey is None else log.get(xkey)
                if x is None or len(x) != len(y):
                    continue
                y = np.asarray(y)
                if y.ndim == 2:      # one curve per column (the feet's contact forces)
                    for i in range(y.shape[1]):
                        a.plot(x, y[:, i], label=f"{label} {i}")
                else:
                    a.plot(x, y, "x" if xkey else "-", label=label)
            a.set(xlabel=xl, ylabel=yl, title=title)
            if a.lines:
                a.legend()
        fig.tight_layout()
        fig.savefig(path)
        plt.close(fig)
        return path
