"""Synthetic replay batches in the make_batch layout, built directly in HBM.

Layout contract: handyrl/train.py:33-133, for
turn-based two-player training without opponent observation
(turn_based_training=True, observation=False; Pp = 1):

    observation (B,T,1,*obs)  policy (B,T,1,A)  action (B,T,1,1) int64
    value/reward/return (B,T,P,1)  outcome (B,1,P,1)  episode_mask (B,T,1,1)
    turn_mask/observation_mask (B,T,P,1)  action_mask (B,T,1,A)  progress (B,T,1)

Generator: per-row valid length L ~ U[5, T]; alternating
turn player; omask = tmask; ~30% of actions illegal (action 0 always legal)
masked with 1e32; behaviour logits N(0,1) minus the mask; actions uniform
over legal ones; zero-sum outcome in {-1, 0, 1}; rewards and returns 0;
progress = (t+1)/L; Bernoulli(0.5) observation planes.  Padding beyond L
follows make_batch: masks 0, action_mask 1e32, progress 1, value = outcome.
"""

import torch


def tictactoe_batch(B, T, device, seed=0, obs_shape=(3, 3, 3), A=9, P=2, min_len=5, illegal_p=0.3):
    g = torch.Generator(device=device).manual_seed(seed)
    dev = device

    def rand(*shape):
        return torch.rand(*shape, device=dev, generator=g)

    lo = min(min_len, T)
    L = torch.randint(lo, T + 1, (B, 1), device=dev, generator=g)
    t = torch.arange(T, device=dev).view(1, T)
    valid = (t < L).float()                                       # (B,T)
    first = torch.randint(0, P, (B, 1), device=dev, generator=g)
    turn = (t + first) % P                                        # alternating turn player
    onehot = torch.nn.functional.one_hot(turn, P).float() * valid.unsqueeze(-1)   # (B,T,P)
    tmask = onehot.unsqueeze(-1)                                  # (B,T,P,1)

    illegal = (rand(B, T, 1, A) < illegal_p)
    illegal[..., 0] = False
    amask = illegal.float() * 1e32
    amask = torch.where(valid.view(B, T, 1, 1) > 0, amask, torch.full_like(amask, 1e32))
    logits = torch.randn(B, T, 1, A, device=dev, generator=g)
    policy = (logits - amask) * valid.view(B, T, 1, 1)            # padded policy rows are 0

    # uniform over legal actions
    score = rand(B, T, 1, A).masked_fill(illegal, -1.0)
    action = score.argmax(-1, keepdim=True)                       # (B,T,1,1) int64
    action = action * valid.view(B, T, 1, 1).long()

    if P == 2:
        o0 = torch.randint(-1, 2, (B, 1, 1, 1), device=dev, generator=g).float()
        outcome = torch.cat([o0, -o0], dim=2)                     # (B,1,2,1) zero-sum
    else:   # rank outcomes of a 4-player game, one per trained player
        outcome = (torch.randint(0, 4, (B, 1, P, 1), device=dev, generator=g).float() * 2 - 3) / 3
    values = torch.tanh(torch.randn(B, T, P, 1, device=dev, generator=g)) * tmask
    values = values + outcome * (1 - valid.view(B, T, 1, 1))      # padded with the outcome

    progress = ((t + 1).float() / L.float()).clamp(max=1.0)
    progress = torch.where(valid > 0, progress, torch.ones_like(progress)).unsqueeze(-1)

    obs = (rand(B, T, 1, *obs_shape) < 0.5).float() * valid.view(B, T, 1, *([1] * len(obs_shape)))

    zeros = torch.zeros(B, T, P, 1, device=dev)
    return {
        'observation': obs,
        'policy': policy.contiguous(), 'value': values.contiguous(),
        'action': action.contiguous(), 'outcome': outcome.contiguous(),
        'reward': zeros, 'return': zeros.clone(),
        'episode_mask': valid.view(B, T, 1, 1).contiguous(),
        'turn_mask': tmask.contiguous(), 'observation_mask': tmask.clone(),
        'action_mask': amask.contiguous(),
        'progress': progress.contiguous(),
    }


def geister_batch(B, T, device, seed=0, P=2, min_len=5):
    """C3 Geister batch: observation {'board': (B,T,1,7,6,6), 'scalar': (B,T,1,18)}, A = 214.

    Same generator as tictactoe_batch (the Bernoulli board planes come from
    it); the scalar features are Bernoulli(0.5) too, zero on padded steps.
    """
    batch = tictactoe_batch(B, T, device, seed=seed, obs_shape=(7, 6, 6), A=214, P=P, min_len=min_len)
    g = torch.Generator(device=device).manual_seed(seed + 1)
    valid = batch['episode_mask'].view(B, T, 1, 1)
    scalar = (torch.rand(B, T, 1, 18, device=device, generator=g) < 0.5).float() * valid
    batch['observation'] = {'board': batch['observation'], 'scalar': scalar.contiguous()}
    return batch


def geese_batch(B, T, device, seed=0, min_len=5):
    """C4 Hungry Geese batch, solo training (turn_based_training=False: make_batch keeps one random
    player per window, train.py:57-58, so P = Pp = 1): observation (B,T,1,17,7,11), A = 4, every
    action legal (hungry_geese.py:187-189), rank outcomes in {-1, -1/3, 1/3, 1}."""
    batch = tictactoe_batch(B, T, device, seed=seed, obs_shape=(17, 7, 11), A=4, P=1, min_len=min_len,
                            illegal_p=0.0)
    # sparse planes like the real observation (hungry_geese.py:211-230: heads, tails, bodies,
    # previous heads, food): plane 0 is the trained goose's head, one cell
    g = torch.Generator(device=device).manual_seed(seed + 1)
    valid = batch['episode_mask'].view(B, T, 1, 1, 1, 1)
    obs = (torch.rand(B, T, 1, 17, 7, 11, device=device, generator=g) < 0.06).float()
    head = torch.randint(0, 77, (B, T, 1), device=device, generator=g)
    obs[:, :, :, 0] = torch.nn.functional.one_hot(head, 77).float().view(B, T, 1, 7, 11)
    batch['observation'] = (obs * valid).contiguous()
    return batch


def geese_args(T, batch_size=None):
    """Learner arguments of config C4: solo (non-turn-based) training, UPGO policy target."""
    args = default_args(T, batch_size)
    args['turn_based_training'] = False
    return args


def default_args(T, batch_size=None):
    """config.yaml train_args for the learner (config.yaml:9-31), TicTacToe-style."""
    return {
        'turn_based_training': True, 'observation': False,
        'gamma': 0.8, 'forward_steps': T, 'compress_steps': 4,
        'entropy_regularization': 1.0e-1, 'entropy_regularization_decay': 0.1,
        'batch_size': batch_size or 64, 'lambda': 0.7,
        'policy_target': 'UPGO', 'value_target': 'VTRACE',
    }
