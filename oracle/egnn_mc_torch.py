"""TEST INFRASTRUCTURE (CPU baseline only; never imported by the product path).

A float64 torch restatement of EGNNMultiChannel's forward (models/egnn_mc/egnn_mc.py:45-295,
with the inputs of dataloaders/egnn_mc_n_body_dataloader.py:8-56) for timing the reference-style
training step (trainer.py:233-358: forward, loss.backward(), optimizer.step()) on host cores in
bench.py --model egnn_mc_train.  Parameters come from a native module's state_dict (same names).
Its gradients are pinned by the same fixture as the native backward (tests/golden/egnn_mc_grad.npz,
tests/test_egnn_mc.py)."""
import torch


def _silu(x):
    return x * torch.sigmoid(x)


def _lin(P, name, x, bias=True):
    y = x @ P[name + ".weight"].T
    return y + P[name + ".bias"] if bias else y


def forward(P, pos, vel, mass, B, N, num_layers, num_heads=2, norm_diff=True, use_tanh=True, recurrent=True,
            coords_weight=1.0):
    """pos / vel [B N, 3], mass [B N, 1] -> pred [B N, 3 num_heads]."""
    ii = torch.arange(N).repeat_interleave(N - 1)
    jj = torch.tensor([j for i in range(N) for j in range(N) if j != i])
    off = (torch.arange(B) * N).repeat_interleave(N * (N - 1))
    row, col = ii.repeat(B) + off, jj.repeat(B) + off
    d = pos[row] - pos[col]
    d2 = (d ** 2).sum(1, keepdim=True)
    dh = d / torch.sqrt(d2).clamp_min(1e-12)
    ea = torch.cat([mass[row] * mass[col], (vel[row] * dh).sum(1, keepdim=True),
                    (vel[col] * dh).sum(1, keepdim=True), d2], 1)
    x = torch.cat([vel.norm(dim=1, keepdim=True), mass], 1)
    h = _lin(P, "embedding", x)
    coord = pos
    V = B * N
    for l in range(num_layers):
        p = f"layers.{l}."
        diff = coord[row] - coord[col]
        radial = (diff ** 2).sum(1, keepdim=True)
        if norm_diff:
            diff = diff / torch.sqrt(radial).clamp_min(1.0)
        ef = _silu(_lin(P, p + "edge_mlp.2", _silu(_lin(P, p + "edge_mlp.0", torch.cat([h[row], h[col], radial, ea], 1)))))
        c = _lin(P, p + "coord_mlp.2", _silu(_lin(P, p + "coord_mlp.0", ef)), bias=False)
        if use_tanh:
            c = torch.tanh(c)
        trans = torch.clamp(diff * c, -100.0, 100.0)
        coord = coord + trans.reshape(V, N - 1, 3).mean(1) * coords_weight
        coord = coord + _lin(P, p + "coord_mlp_vel.2", _silu(_lin(P, p + "coord_mlp_vel.0", h))) * vel
        agg = ef.reshape(V, N - 1, -1).mean(1)
        hn = _lin(P, p + "node_mlp.2", _silu(_lin(P, p + "node_mlp.0", torch.cat([h, agg], 1))))
        h = h + hn if recurrent else hn
    hin = torch.cat([h, coord - pos, vel], 1)
    outs = [_lin(P, f"heads.{t}.net.4", _silu(_lin(P, f"heads.{t}.net.2", _silu(_lin(P, f"heads.{t}.net.0", hin)))))
            for t in range(num_heads)]
    return torch.cat(outs, 1)
