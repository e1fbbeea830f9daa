"""RL reward-price agent, host side (reference `dragg/agent.py:42-282`).

The north star keeps the agent on the host: it is a few dozen flops per timestep on
~50-dimensional feature vectors, against a community solve of 10^4-10^5 homes on the GPU.
What the agent needs from the community -- the aggregate load, its forecast, the setpoint,
and candidate-price rollouts -- comes from `dragg_amd.runner.Aggregator` (`rl_step`,
`rl_forecast`, `collect_data`), i.e. from device-resident solves.

`RLAgent` restates the reference's abstract base: linear-Gaussian policy over the
state basis, linear critic over the state-action basis (optionally twin), experience
replay with a ridge fit, eligibility-trace policy update.  The reference leaves
`calc_state` and `reward` abstract and ships no concrete agent or driver at v1 (the RL
case of `Aggregator.run` does not exist, `rl.utility.action_space` is absent from its
config, agent.py:75); `SetpointAgent` below is this build's concrete agent -- its state and
reward definitions are ours, documented as such ("parity unpinned").
"""
import random
from abc import ABC, abstractmethod

import numpy as np


def ridge_fit(X, y, alpha=0.01):
    """sklearn `Ridge(alpha).fit(X, y).coef_` (fit_intercept=True, dense Cholesky solve) as used
    at agent.py:200-203: centre X and y, solve (XcᵀXc + αI) w = Xcᵀyc."""
    X = np.asarray(X, dtype=float)
    y = np.asarray(y, dtype=float)
    Xc = X - X.mean(axis=0)
    yc = y - y.mean()
    A = Xc.T @ Xc + alpha * np.eye(X.shape[1])
    return np.linalg.solve(A, Xc.T @ yc)


class RLAgent(ABC):
    """agent.py:42-282.  `parameters`: {alpha, beta, batch_size, twin_q, epsilon} (agent.py:78-86);
    `config`: the run's config dict (its `rl.utility.action_space` is required, as at agent.py:75)."""

    def __init__(self, parameters, config, rl_log=None, rng=None):
        self.config = config
        self.actionspace = config["rl"]["utility"]["action_space"]   # KeyError like agent.py:75
        self.theta_mu = None
        self.theta_q = None
        self.prev_state = None
        self.state = None
        self.next_state = None
        self.action = None
        self.next_action = None
        self.memory = []
        self.cumulative_reward = 0
        self.average_reward = 0
        self.mu = 0
        self.rla_log = rl_log
        self.i = 0
        self.z_theta_mu = 0
        self.lam_theta = 0.01
        # scipy.stats.norm.rvs / np.random.normal draw from numpy's global RandomState
        # (agent.py:163, 189); `rng` may pin it
        self.rng = rng if rng is not None else np.random.mtrand._rand
        self.rl_data = {}
        self.set_rl_data()
        self._set_parameters(parameters)

    @abstractmethod
    def calc_state(self, env):
        pass

    @abstractmethod
    def reward(self):
        pass

    # agent.py:78-86
    def _set_parameters(self, params):
        self.ALPHA_q = params["alpha"]
        self.ALPHA_mu = params["alpha"]
        self.ALPHA_w = params["alpha"] * 2
        self.ALPHA_r = params["alpha"] * 2 ** 2
        self.BETA = params["beta"]
        self.BATCH_SIZE = params["batch_size"]
        self.TWIN_Q = params["twin_q"]
        self.SIGMA = params["epsilon"]

    # agent.py:88-95: features (1, e, e²) ⊗ (1, f, f²) ⊗ (1, sin, cos), constant dropped twice
    @staticmethod
    def state_basis(state):
        e = np.array([1, state["fcst_error"], state["fcst_error"] ** 2])
        f = np.array([1, state["forecast_trend"], state["forecast_trend"] ** 2])
        tod = 2 * np.pi * state["time_of_day"]
        tb = np.array([1, np.sin(tod), np.cos(tod)])
        phi = np.outer(e, f).flatten()[1:]
        return np.outer(phi, tb).flatten()[1:]

    # agent.py:97-110
    @staticmethod
    def state_action_basis(state, action):
        ab = np.array([1, action, action ** 2])
        db = np.array([1, state["delta_action"], state["delta_action"] ** 2])
        tod = 2 * np.pi * state["time_of_day"]
        tb = np.array([1, np.sin(tod), np.cos(tod)])
        e = np.array([1, state["fcst_error"], state["fcst_error"] ** 2])
        f = np.array([1, state["forecast_trend"], state["forecast_trend"] ** 2])
        v = np.outer(f, ab).flatten()[1:]
        w = np.outer(e, ab).flatten()[1:]
        z = np.outer(e, db).flatten()[1:]
        phi = np.concatenate((v, w, z))
        return np.outer(phi, tb).flatten()[1:]

    # agent.py:124-127
    def memorize(self):
        if self.state and self.action:
            self.memory.append({"state": self.state, "action": self.action, "reward": self.r,
                                "next_state": self.next_state})

    # agent.py:129-149
    def train(self, env):
        self.next_state = self.calc_state(env)
        if not self.state:
            self.state = self.next_state
        if not self.next_action:
            self.next_action = 0
        self.action = self.next_action
        self.r = self.reward()
        self.xu_k = self.state_action_basis(self.state, self.action)
        self.next_action = self.get_policy_action(self.next_state)
        self.xu_k1 = self.state_action_basis(self.next_state, self.next_action)
        self.memorize()
        self.update_qfunction()
        self.update_policy()
        self.record_rl_data()
        self.state = self.next_state
        return self.next_action

    # agent.py:151-165
    def get_policy_action(self, state):
        x_k = self.state_basis(state)
        if self.theta_mu is None:
            self.theta_mu = np.zeros(len(x_k))
        self.mu = self.theta_mu @ x_k
        return self.rng.normal(loc=self.mu, scale=self.SIGMA)

    # agent.py:178-187 (process_exp; parse_exp is the same plus xu_k)
    def process_exp(self, exp):
        u1 = self.get_policy_action(exp["next_state"])
        xu_k1 = self.state_action_basis(exp["next_state"], u1)
        q_k1 = min(self.theta_q[:, i] @ xu_k1 for i in range(self.theta_q.shape[1]))
        return exp["reward"] + self.BETA * q_k1

    # agent.py:189-204.  The replay batch is processed in-process (the reference forks a
    # ProcessPool for ~BATCH_SIZE dot products).
    def update_qfunction(self):
        if self.TWIN_Q:
            self.i = (self.i + 1) % 2
        if self.theta_q is None:
            n = len(self.state_action_basis(self.state, self.action))
            m = 2 if self.TWIN_Q else 1
            self.theta_q = self.rng.normal(0, 0.3, (n, m))
        self.q_predicted = self.theta_q[:, self.i] @ self.xu_k
        self.q_observed = self.r + self.BETA * self.theta_q[:, self.i] @ self.xu_k1
        if len(self.memory) > self.BATCH_SIZE:
            batch = random.sample(self.memory, self.BATCH_SIZE)
            batch_y = np.array([self.process_exp(e) for e in batch])
            batch_phi = np.array([self.state_action_basis(e["state"], e["action"]) for e in batch])
            temp_theta = ridge_fit(batch_phi, batch_y, 0.01)
            # flatten() of a twin critic has 2n entries: numpy raises here exactly as the
            # reference does (agent.py:204)
            self.theta_q[:, self.i] = self.ALPHA_q * temp_theta + (1 - self.ALPHA_q) * self.theta_q.flatten()

    # agent.py:206-224
    def update_policy(self):
        x_k = self.state_basis(self.state)
        delta = np.clip(self.q_predicted - self.q_observed, -1, 1)
        self.average_reward += self.ALPHA_r * delta
        self.cumulative_reward += self.r
        self.mu = self.theta_mu @ x_k
        self.mu = np.clip(self.mu, self.actionspace[0], self.actionspace[1])
        grad_pi_mu = (self.SIGMA ** 2) * (self.action - self.mu) * x_k
        self.z_theta_mu = self.lam_theta * self.z_theta_mu + grad_pi_mu
        self.theta_mu += self.ALPHA_mu * delta * self.z_theta_mu

    # agent.py:226-251
    def set_rl_data(self):
        for k in ("theta_q", "theta_mu", "phi", "q_obs", "q_pred", "action", "q_tables", "average_reward",
                  "cumulative_reward", "reward", "mu"):
            self.rl_data[k] = []

    def record_rl_data(self):
        d = self.rl_data
        d["theta_q"].append(self.theta_q[:, self.i].flatten().tolist())
        d["theta_mu"].append(self.theta_mu.flatten().tolist())
        d["q_obs"].append(float(self.q_observed))
        d["q_pred"].append(float(self.q_predicted))
        d["action"].append(float(self.action))
        d["average_reward"].append(float(self.average_reward))
        d["cumulative_reward"].append(float(self.cumulative_reward))
        d["reward"].append(float(self.r))
        d["mu"].append(float(self.mu))

    # agent.py:253-264
    def record_parameters(self):
        self.rl_data["parameters"] = {"alpha_q": self.ALPHA_q, "alpha_mu": self.ALPHA_mu, "alpha_w": self.ALPHA_w,
                                      "alpha_r": self.ALPHA_r, "beta": self.BETA, "batch_size": self.BATCH_SIZE,
                                      "twin_q": self.TWIN_Q, "sigma": self.SIGMA}

    def write_rl_data(self, output_dir):
        import json
        import os
        with open(os.path.join(output_dir, f"{self.name}_agent-results.json"), "w+") as f:
            json.dump(self.rl_data, f, indent=4)


class SetpointAgent(RLAgent):
    """This build's concrete agent (not in the reference, which leaves calc_state / reward
    abstract): it steers the community's forecast load toward the aggregator's setpoint.

    state: fcst_error = (forecast_load - setpoint) / setpoint, forecast_trend = relative change
    of the forecast load, time_of_day in [0, 1), delta_action = last action change;
    reward = -fcst_error².  The action is the reward price × `action_scale` (README.md:73)."""

    name = "setpoint"

    def __init__(self, parameters, config, rl_log=None, rng=None):
        super().__init__(parameters, config, rl_log, rng)
        self.action_scale = float(config["rl"]["utility"].get("action_scale", 100.0))
        self._err = 0.0
        self._prev_action = 0.0

    def calc_state(self, env):
        sp = env.agg_setpoint if env.agg_setpoint else 1.0
        self._err = (env.forecast_load - sp) / sp
        prev = env.prev_forecast_load if env.prev_forecast_load else 1.0
        trend = (env.forecast_load - prev) / prev
        env.prev_forecast_load = env.forecast_load
        steps_per_day = 24 * env.dt
        a = float(self.action) if self.action is not None else 0.0
        d = a - self._prev_action
        self._prev_action = a
        return {"fcst_error": self._err, "forecast_trend": trend,
                "time_of_day": (env.timestep % steps_per_day) / steps_per_day, "delta_action": d}

    def reward(self):
        return -self._err ** 2

    def act(self, env):
        """policy(aggregator) -> reward price for `Aggregator.run_rl_agg`."""
        a = float(np.clip(self.train(env), self.actionspace[0], self.actionspace[1]))
        return a / self.action_scale


def agent_policy(aggregator):
    """The agent a `run_rl_agg = true` config runs with: rl.parameters (README.md:58-63)."""
    p = aggregator.config["rl"]["parameters"]
    agent = SetpointAgent({"alpha": p["learning_rate"], "beta": p["discount_factor"], "batch_size": p["batch_size"],
                           "twin_q": p["twin_q"], "epsilon": p["exploration_rate"]}, aggregator.config)
    return agent.act
