"""MuZero agent drop-in (reference: Muzero.py:13-323, `Muzero`) -- SURVEY.md section 8f rank 3.

Same constructor and `training_loop(n_loops, min_replay_size, print_acc)` as the reference, so
`training_main.py` can construct it unchanged.  What runs where on the MI355X:
  * self-play (`_play_game`): every search is one fused libmzh kernel launch (mcts.MCTS) and the
    environment step is the reference's (selfplay.play_game); with selfplay="batched" the
    n_ep_x_loop episodes of a loop play in lockstep -- one search launch and one env-kernel launch
    per step for all of them (selfplay.BatchedSelfPlay), each episode an agent whose MinMaxStats
    starts from the MCTS instance's, then the reference's per-episode bookkeeping
    (selfplay.episode_records) and buffer filter.  With n_ep_x_loop > 1 that is NOT the
    reference's schedule (one MinMaxStats chain through the episodes in order, Muzero.py:55; other
    per-step draw interleaving): a RuntimeWarning says so, and "sequential" (the default) is the
    parity mode;
  * the replay buffer keeps its transitions on the training device (buffer.Buffer);
  * the update (`_update`, Muzero.py:209-274): the 5-step unrolled loss of the reference -- the
    same torch operations in the same order (represent, prediction/dynamics per unroll step,
    0.5 gradient scaling of the dynamics latent, MSE value / reward and cross-entropy policy terms,
    importance weights, 1/unroll gradient scaling, Adam) -- on PyTorch-ROCm.  After each update
    the search engine repacks the weights (networks.engine_for tracks parameter versions).
"""
import ctypes
import logging
import math
import warnings

import numpy as np
import torch
import torch.nn.functional as F
from torch.autograd.graph import increment_version

from .buffer import Buffer
from .mcts import MCTS
from .networks import MuZeroNet
from .selfplay import BatchedSelfPlay, episode_records, play_game
from .utils import adjust_temperature, organise_transitions


class Muzero:
    def __init__(self, env, s_space_size, n_action, discount, dirichlet_alpha, n_mcts_simulations, unroll_n_steps,
                 batch_s, TD_return, n_TD_step, lr, buffer_size, priority_replay, device, n_ep_x_loop=1,
                 n_update_x_loop=1, update_impl="torch", selfplay="sequential", device_sampling=None):
        self.dev = device
        self.env = env
        self.n_ep_x_loop = n_ep_x_loop  # episodes collected per training loop
        self.discount = discount
        self.n_action = n_action
        self.unroll_n_steps = unroll_n_steps
        self.n_update_x_loop = n_update_x_loop  # updates per training loop
        self.batch_s = batch_s
        self.TD_return = TD_return
        self.n_step = n_TD_step
        self.mcts = MCTS(discount=discount, root_dirichlet_alpha=dirichlet_alpha, n_simulations=n_mcts_simulations,
                         batch_s=batch_s, device=device)
        self.networks = MuZeroNet(rpr_input_s=s_space_size, action_s=n_action, lr=lr, TD_return=TD_return,
                                  device=device).to(device)
        # device_sampling (not in the reference's signature): the prioritised draw and the priority
        # write-back on the device (buffer.Buffer); by default with the fused update on a GPU
        if device_sampling is None:
            device_sampling = update_impl == "fused" and bool(priority_replay) and torch.device(device).type == "cuda"
        self.buffer = Buffer(buffer_size, unroll_n_steps, d_state=s_space_size, n_action=n_action, device=device,
                             device_sampling=device_sampling)
        self.priority_replay = priority_replay
        # update_impl (not in the reference's signature): "torch" = the reference's op sequence,
        # "graph" = that sequence replayed as one HIP graph (GraphedUpdate), "fused" = the two-kernel
        # HIP update of libmzh (FusedUpdate)
        if update_impl not in ("torch", "graph", "fused"):
            raise ValueError(f"update_impl must be 'torch', 'graph' or 'fused', not {update_impl!r}")
        self._graphed = {"torch": None, "graph": GraphedUpdate, "fused": FusedUpdate}[update_impl]
        if self._graphed is not None:
            self._graphed = self._graphed(self)
        # selfplay (not in the reference's signature): "sequential" = one episode after another as
        # Muzero._play_game runs them; "batched" = a loop's n_ep_x_loop episodes in lockstep
        if selfplay not in ("sequential", "batched"):
            raise ValueError(f"selfplay must be 'sequential' or 'batched', not {selfplay!r}")
        if selfplay == "batched" and n_ep_x_loop > 1:
            # not the reference's algorithm: the reference threads ONE MinMaxStats through its
            # episodes in order (Muzero.py:55) and interleaves the per-step draws differently
            warnings.warn("Muzero(selfplay='batched') with n_ep_x_loop > 1 plays the loop's episodes in lockstep, "
                          "each from the same MinMaxStats (the union kept afterwards) with its own draw order: "
                          "not the reference's sequential schedule; use selfplay='sequential' for parity runs",
                          RuntimeWarning, stacklevel=2)
        self.selfplay = selfplay

    # ------------------------------------------------------------------ Muzero.py:81-151
    def training_loop(self, n_loops, min_replay_size, print_acc=50):
        logging.info("Training started \n")
        accuracy, tot_accuracy = [], []
        value_loss, rwd_loss, pi_loss = [], [], []
        for n in range(1, n_loops):
            ep_steps = []
            if self.selfplay == "batched":
                episodes = self._play_games(self.n_ep_x_loop, episode=n * self.n_ep_x_loop, deterministic=False)
            else:
                episodes = (self._play_game(episode=n * self.n_ep_x_loop, deterministic=False)
                            for _ in range(self.n_ep_x_loop))
            for steps, states, rwds, actions, pi_probs, returns, priorities in episodes:
                ep_steps.append(steps)
                if returns[-1, 0] > 0:  # only successful episodes enter the buffer
                    self.buffer.add(states, rwds, actions, pi_probs, returns, priorities)
            accuracy.append(sum(ep_steps) / self.n_ep_x_loop)
            if len(self.buffer) > min_replay_size:
                for _ in range(self.n_update_x_loop):
                    if self.priority_replay:
                        states, rwds, actions, pi_probs, returns, indx, w = self.buffer.priority_sample(self.batch_s)
                    else:
                        states, rwds, actions, pi_probs, returns = self.buffer.uniform_sample(self.batch_s)
                        indx, w = None, None
                    new_prio, v_loss, r_loss, p_loss = self._update(states, rwds, actions, pi_probs, returns, w)
                    self.buffer.update_priorities(indx, new_prio)
                value_loss.append(v_loss)
                rwd_loss.append(r_loss)
                pi_loss.append(p_loss)
            if n * self.n_ep_x_loop % print_acc == 0:
                mean_acc = sum(accuracy) / print_acc
                logging.info("Loop %s | steps %.3f | V %.3f | rwd %.3f | Pi %.3f", n, mean_acc,
                             sum(value_loss) / print_acc, sum(rwd_loss) / print_acc, sum(pi_loss) / print_acc)
                tot_accuracy.append(mean_acc)
                accuracy = []
                value_loss, rwd_loss, pi_loss = [], [], []
        return tot_accuracy

    # ------------------------------------------------------------------ Muzero.py:153-207
    def _play_game(self, episode, deterministic=False):
        return play_game(self.env, self.mcts, self.networks, episode, deterministic, discount=self.discount,
                         TD_return=self.TD_return, n_step=self.n_step, unroll_n_steps=self.unroll_n_steps,
                         n_action=self.n_action)

    def _play_games(self, n_games, episode, deterministic=False):
        """n_games episodes from env.reset()'s start in lockstep (BatchedSelfPlay): each one an
        agent whose MinMaxStats starts from this MCTS instance's; afterwards the instance keeps
        the union (max of the maxima, min of the minima).  Draws come from the global NumPy stream
        (for n_games = 1 exactly the draws of _play_game).  Returns _play_game's tuple per episode."""
        env, mm = self.env, self.mcts.min_max_stats
        sp = BatchedSelfPlay(self.networks, env.discs, env.max_steps, int(self.mcts.n_simulations),
                             discount=self.discount, dirichlet_alpha=self.mcts.root_dirichlet_alpha,
                             root_exploration_eps=self.mcts.root_exploration_eps, goal_peg=env.goal[0],
                             np1_ucb=self.mcts.np1_ucb)
        res = sp.play([env.init_state_idx] * n_games, temperature=adjust_temperature(episode),
                      deterministic=deterministic, legacy_rng=True,
                      minmax=[[mm.maximum, mm.minimum]] * n_games, record_obs=True)
        fin = res["minmax"].cpu().numpy()
        mm.maximum, mm.minimum = float(fin[:, 0].max()), float(fin[:, 1].min())
        return episode_records(res, discount=self.discount, TD_return=self.TD_return, n_step=self.n_step,
                               unroll_n_steps=self.unroll_n_steps, n_action=self.n_action)

    # ------------------------------------------------------------------ Muzero.py:209-274
    def _update(self, states, rwds, actions, pi_probs, returns, priority_w):
        if self._graphed is not None:
            return self._graphed(states, rwds, actions, pi_probs, returns, priority_w)
        net, U = self.networks, self.unroll_n_steps
        v_terms, r_terms, p_terms, pred_values_t = unrolled_losses(net, states, rwds, actions, pi_probs, returns, U,
                                                                    self.dev)
        loss = v_terms + r_terms + p_terms
        new_priorities = None
        if priority_w is not None:
            loss = loss * priority_w.detach()  # importance-sampling weights of the prioritised sample
            with torch.no_grad():
                pred0 = torch.stack(pred_values_t, dim=1).squeeze(-1)[:, 0]
                new_priorities = (pred0 - returns[:, 0]).abs().cpu().numpy()
        loss = loss.mean()
        loss.register_hook(lambda grad: grad * (1 / U))  # loss scaled by 1/unroll_steps (through the hook)
        net.update(loss)
        return new_priorities, v_terms.mean().detach(), r_terms.mean().detach(), p_terms.mean().detach()

    def organise_transitions(self, episode_state, episode_rwd, episode_action, episode_piProb, episode_returns):
        """Muzero.py:276-323"""
        return organise_transitions(episode_state, episode_rwd, episode_action, episode_piProb, episode_returns,
                                    self.unroll_n_steps, self.n_action)


def unrolled_losses(net, states, rwds, actions, pi_probs, returns, unroll_n_steps, device):
    """Per-sample value / reward / policy loss sums over the unrolled steps (Muzero.py:213-245), in
    the reference's operation order: h = represent(s); for each step t: prediction(h), then
    dynamics(h, onehot(a_t)) with the new latent's gradient halved, then the three loss terms."""
    v_sum = r_sum = p_sum = 0
    pred_values_t = []
    h = net.represent(states)
    for t in range(unroll_n_steps):
        pi_logits, values = net.prediction(h)
        onehot = F.one_hot(actions[:, t], num_classes=net.num_actions).squeeze().to(device, dtype=torch.long)
        h, pred_rwds = net.dynamics(h, onehot)
        h.register_hook(lambda grad: grad * 0.5)  # scale the dynamics gradient by 0.5
        v_sum += F.mse_loss(values.squeeze(), returns[:, t], reduction="none")
        r_sum += F.mse_loss(pred_rwds.squeeze(), rwds[:, t], reduction="none")
        p_sum += F.cross_entropy(pi_logits, pi_probs[:, t], reduction="none")  # logits in, softmax inside
        pred_values_t.append(values)
    return v_sum, r_sum, p_sum, pred_values_t


class GraphedUpdate:
    """`Muzero._update` captured once as a HIP graph and replayed per batch.

    At the reference's batch (256 transitions, 5 unroll steps, 256-wide MLPs) one update is a few
    hundred small kernels, so on the GPU it is bound by launch overhead, not by the GEMMs.  The
    graph holds the same torch operations as the eager `_update` (same order, same hooks); the
    only change is Adam's `capturable=True` form (step count and bias corrections kept on the
    device, so fp32 rather than Python-float step sizes: ulp-level differences).  Inputs are
    copied into static buffers, so the batch size and the prioritised/uniform choice are fixed
    at capture time (the first call).  Warm-up iterations run on a snapshot that is restored
    before capture, so the graph's first replay is the first real update.
    """

    def __init__(self, mz, warmup=3):
        if not str(mz.dev).startswith("cuda"):
            raise RuntimeError("graph_update needs a GPU device")
        self.mz = mz
        self.warmup = warmup
        self.graph = None
        net = mz.networks
        old = net.optimiser
        net.optimiser = opt_like(old, capturable=True, fused=True)

    def _capture(self, states, rwds, actions, pi_probs, returns, priority_w):
        mz, net, U = self.mz, self.mz.networks, self.mz.unroll_n_steps
        self.prio = priority_w is not None
        self.static_in = [t.detach().clone() for t in (states, rwds, actions, pi_probs, returns)]
        self.static_w = priority_w.detach().clone() if self.prio else None
        params = [p.detach().clone() for p in net.parameters()]
        opt_state = copy_opt_state(net.optimiser)

        def body():
            v, r, p, pred_values_t = unrolled_losses(net, *self.static_in, U, mz.dev)
            loss = v + r + p
            newp = None
            if self.prio:
                loss = loss * self.static_w
                with torch.no_grad():
                    newp = (torch.stack(pred_values_t, dim=1).squeeze(-1)[:, 0] - self.static_in[4][:, 0]).abs()
            loss = loss.mean()
            loss.register_hook(lambda grad: grad * (1 / U))
            loss.backward()
            net.optimiser.step()
            return newp, v.mean().detach(), r.mean().detach(), p.mean().detach()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                net.optimiser.zero_grad(set_to_none=True)
                body()
        torch.cuda.current_stream().wait_stream(side)
        with torch.no_grad():  # undo the warm-up updates
            for q, p0 in zip(net.parameters(), params):
                q.copy_(p0)
            restore_opt_state(net.optimiser, opt_state)
        net.optimiser.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = body()

    def __call__(self, states, rwds, actions, pi_probs, returns, priority_w):
        if self.graph is None:
            self._capture(states, rwds, actions, pi_probs, returns, priority_w)
        else:
            if (priority_w is not None) != self.prio or states.shape != self.static_in[0].shape:
                raise ValueError("graph_update: batch shape / sampling mode changed after capture")
            for dst, src in zip(self.static_in, (states, rwds, actions, pi_probs, returns)):
                dst.copy_(src)
            if self.prio:
                self.static_w.copy_(priority_w)
        self.graph.replay()
        newp, v, r, p = self.out
        return (newp.cpu().numpy() if newp is not None else None), v.clone(), r.clone(), p.clone()


def opt_like(old, **overrides):
    """a torch.optim.Adam with `old`'s parameters, hyper-parameters and state, plus `overrides`"""
    groups = [{k: v for k, v in g.items() if k != "params"} for g in old.param_groups]
    params = [p for g in old.param_groups for p in g["params"]]
    d = dict(groups[0])
    d.update(overrides)
    new = torch.optim.Adam(params, **{k: d[k] for k in ("lr", "betas", "eps", "weight_decay", "amsgrad",
                                                        "capturable", "fused") if k in d})
    st = old.state_dict()
    if st["state"]:
        for s in st["state"].values():  # capturable Adam keeps the step count on the parameter's device
            s["step"] = torch.as_tensor(float(s["step"]), dtype=torch.float32, device=params[0].device)
        st["param_groups"][0].update(overrides)
        new.load_state_dict(st)
    return new


def copy_opt_state(o):
    return {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in s.items()} for p, s in o.state.items()}


def restore_opt_state(o, saved):
    for p in list(o.state.keys()):
        if id(p) in saved:
            for k, v in saved[id(p)].items():
                if torch.is_tensor(o.state[p][k]) and torch.is_tensor(v):
                    o.state[p][k].copy_(v)
                else:
                    o.state[p][k] = v
        else:  # state created by the warm-up only: back to "no step taken yet", in place
            for k, v in o.state[p].items():
                if torch.is_tensor(v):
                    v.zero_()


class FusedUpdate:
    """`Muzero._update` + Adam as libmzh's fused HIP training update (csrc/mzh_train.hip).

    Launch 1 runs, per transition, the U-step unrolled forward and the complete backward pass of
    the reference's loss (Muzero.py:213-265) in one workgroup; launch 2 forms every weight gradient
    as a GEMM over the B*U rows on fp32 MFMA and applies torch.optim.Adam's update in place on the
    module's parameters and the optimiser's own state tensors, so `networks.state_dict()` and
    `networks.optimiser.state_dict()` (the checkpoint of training_main.py:93-103) stay the
    reference's.  Adam's step counter and bias corrections are the host-side Python floats torch
    uses.  Results match the torch update to fp32 rounding (other summation orders).
    """

    def __init__(self, mz):
        if not str(mz.dev).startswith("cuda"):
            raise RuntimeError("update_impl='fused' needs a GPU device")
        from . import _lib
        self._lib = _lib
        self.mz = mz
        net = mz.networks
        self.params = list(net.parameters())
        if len(self.params) != 20:
            raise ValueError("fused update expects MuZeroNet's 20 parameter tensors")
        g = net.optimiser.param_groups[0]
        if not isinstance(net.optimiser, torch.optim.Adam) or g["weight_decay"] != 0 or g["amsgrad"] \
                or g.get("maximize", False) or len(net.optimiser.param_groups) != 1:
            raise ValueError("fused update implements plain torch.optim.Adam (no weight decay / amsgrad)")
        self.support = net.support_size
        self.in_dim = self.params[0].shape[1]
        dev = self.params[0].device
        # transposed weight copies [in][out rounded up to 4] (16-byte rows for float4 loads)
        self.wt = [torch.zeros(p.shape[1], (p.shape[0] + 3) // 4 * 4, dtype=torch.float32, device=dev)
                   for p in self.params[0::2]]
        self.scratch = None
        self.B = None
        self._a = None
        self._seen = None  # parameter versions after our own last write

    def _versions(self):
        return tuple((p.data_ptr(), p._version) for p in self.params)

    def _state(self):
        opt = self.mz.networks.optimiser
        for p in self.params:
            st = opt.state[p]
            if len(st) == 0:  # torch.optim.Adam._init_group's lazy state
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return [opt.state[p] for p in self.params]

    def _setup(self, B, device):
        """scratch / outputs for batch size B and the argument block's fixed pointers: parameters,
        transposed copies and the optimiser's moment tensors (re-done when the optimiser's state
        objects change, e.g. after load_state_dict)"""
        L = self._lib
        U = self.mz.unroll_n_steps
        if self.B != B:
            nb = ctypes.c_size_t()
            L.check(L.lib().mzh_train_scratch_bytes(B, U, self.in_dim, self.support, nb), "mzh_train_scratch_bytes")
            self.scratch = torch.empty(nb.value // 4 + 64, dtype=torch.float32, device=device)
            self.row_loss = torch.empty(B, 3, dtype=torch.float32, device=device)
            self.new_prio = torch.empty(B, dtype=torch.float32, device=device)
            self.B = B
        states_ = self._state()
        a = L.TrainArgs()
        a.B, a.U, a.in_dim, a.support, a.rows = B, U, self.in_dim, self.support, 0
        for i, p in enumerate(self.params):
            a.param[i] = p.data_ptr()
        for i, w in enumerate(self.wt):
            a.wt[i] = w.data_ptr()
        for i, st in enumerate(states_):
            a.exp_avg[i] = st["exp_avg"].data_ptr()
            a.exp_avg_sq[i] = st["exp_avg_sq"].data_ptr()
        a.scratch = self.scratch.data_ptr()
        a.scratch_bytes = self.scratch.numel() * 4
        a.row_loss = self.row_loss.data_ptr()
        self._a = a
        # Adam's per-parameter step counters (0-dim host tensors in the optimiser's state): written through
        # NumPy views (one _foreach_add_ over 20 host tensors costs more than the update's launch)
        self._step_views = [st["step"].numpy() for st in states_]
        self._state_key = self._state_identity()

    def _state_identity(self):
        # Optimizer.load_state_dict installs a new state dict: its identity (and size) marks a reload
        opt = self.mz.networks.optimiser
        return id(opt.state), len(opt.state)

    def __call__(self, states, rwds, actions, pi_probs, returns, priority_w):
        L = self._lib
        B = states.shape[0]
        stream = torch.cuda.current_stream().cuda_stream
        if self._a is None or self.B != B or self._state_key != self._state_identity():
            self._setup(B, states.device)
        a = self._a
        if self._seen != self._versions():  # parameters written outside this update: re-transpose
            L.check(L.lib().mzh_train_transpose(a, stream), "mzh_train_transpose")
        g = self.mz.networks.optimiser.param_groups[0]
        beta1, beta2 = g["betas"]
        step = float(self._step_views[0]) + 1.0  # this update's step (written back after the launch)
        a.step_size = g["lr"] / (1 - beta1 ** step)
        a.bc2_sqrt = math.sqrt(1 - beta2 ** step)
        a.beta1, a.beta2, a.eps = beta1, beta2, g["eps"]
        ins = [states.float().contiguous(), rwds.float().contiguous(), actions.long().contiguous(),
               pi_probs.float().contiguous(), returns.float().contiguous()]
        w = priority_w.float().contiguous() if priority_w is not None else None
        a.obs, a.rwds, a.actions, a.pi, a.returns = (t.data_ptr() for t in ins)
        a.weights = w.data_ptr() if w is not None else None
        # with the buffer's device sampling the new priorities stay on the device (a new tensor per
        # update: update_priorities consumes it there); else they go to the host as the reference's do
        on_dev = w is not None and getattr(self.mz.buffer, "device_sampling", False)
        newp_t = torch.empty(B, dtype=torch.float32, device=states.device) if on_dev else self.new_prio
        a.new_prio = newp_t.data_ptr() if w is not None else None
        L.check(L.lib().mzh_train_update(a, stream), "mzh_train_update")
        for v in self._step_views:  # torch.optim.Adam's step += 1 (float32), while the kernels run
            v[...] = step
        increment_version(self.params)  # the kernel wrote the parameters in place: let version trackers know
        self._seen = self._versions()
        means = self.row_loss.mean(0)
        newp = None if w is None else (newp_t if on_dev else newp_t.cpu().numpy())
        return newp, means[0], means[1], means[2]
