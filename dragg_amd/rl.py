"""RL reward-price policies, host side.

The north star keeps the agent on the host: a policy is a few flops per timestep against a
community solve of 10^4-10^5 homes on the GPU.  What a policy needs from the community -- the
aggregate load, its forecast, the setpoint and candidate-price rollouts -- comes from
`dragg_amd.runner.Aggregator` (`rl_step`, `rl_forecast`, `collect_data`), i.e. from
device-resident solves.

The reference's learning agent (`dragg/agent.py`, an abstract actor-critic whose
`calc_state` / `reward` are left to a subclass and which no driver of v1 calls) is out of
scope and is NOT restated here.  It plugs in unchanged through
`policy_from_agent`: any object with the reference agent's `train(env) -> action` method
becomes a `policy(aggregator) -> reward price` for `Aggregator.run_rl_agg`, the aggregator
itself being the `env` it reads.

`SetpointAgent` is this build's own default policy (parity unpinned: the reference ships
none): a discrete PI controller on the relative forecast error against the aggregator's
setpoint (`gen_setpoint`, aggregator.py:677-696), clipped to `rl.utility.action_space`.
"""
import numpy as np


def policy_from_agent(agent, scale=1.0):
    """Wrap a reference-style agent (`train(env) -> action`, agent.py:130-149) as the policy
    `run_rl_agg` calls once per timestep: reward price = action / scale."""
    def policy(aggregator):
        return float(agent.train(aggregator)) / scale
    return policy


class SetpointAgent:
    """Action = kp e + ki Σ e clipped to the action space, e = (forecast - setpoint) /
    setpoint: a forecast above the setpoint raises the reward price (which the homes add to
    TOU, mpc_calc.py:353).  The integral term is clamped to the action space (anti-windup).
    `config["rl"]["utility"]["action_space"]` is required (KeyError, like the reference's agent
    at agent.py:75); `action_scale` maps actions to $/kWh."""

    name = "setpoint"

    def __init__(self, config, kp=1.0, ki=0.1):
        util = config["rl"]["utility"]
        lo, hi = util["action_space"]
        self.lo, self.hi = float(lo), float(hi)
        self.scale = float(util.get("action_scale", 100.0))
        self.kp, self.ki = float(kp), float(ki)
        self.integral = 0.0
        self.history = {"error": [], "action": []}

    def error(self, env):
        sp = env.agg_setpoint if env.agg_setpoint else 1.0
        return (env.forecast_load - sp) / sp

    def train(self, env):
        e = self.error(env)
        if self.ki:
            self.integral = float(np.clip(self.integral + e, self.lo / self.ki, self.hi / self.ki))
        a = float(np.clip(self.kp * e + self.ki * self.integral, self.lo, self.hi))
        self.history["error"].append(e)
        self.history["action"].append(a)
        return a

    def act(self, env):
        """policy(aggregator) -> reward price for `Aggregator.run_rl_agg`."""
        return self.train(env) / self.scale


def agent_policy(aggregator):
    """The policy a `run_rl_agg = true` config runs with: `SetpointAgent`, its gains from the keys of
    its own, `rl.parameters.kp` (default 1.0) and `rl.parameters.ki` (default 0.1).  The reference's
    `rl.parameters.learning_rate` (README.md:58-63) is a learning agent's step size, not a controller
    gain: it is left to an agent wrapped by `policy_from_agent`."""
    p = aggregator.config.get("rl", {}).get("parameters", {}) or {}
    return SetpointAgent(aggregator.config, kp=float(p.get("kp", 1.0)), ki=float(p.get("ki", 0.1))).act
