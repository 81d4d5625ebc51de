"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Torch-CPU restatement of the reference model and training step (the "torch
fp32 reference" for the floating-point kernels).  Same state_dict key names as
the reference, so the deterministic weights of tests/golden_util.py load into
the reference (fixture generation), this oracle, and the HIP model alike.
Pinned by tests/golden/model_s*.npz / tiny_c1.npz (reference outputs, loss
values, every gradient and the post-AdamW parameters).

  geometric_schedule          ref/model/vae_teb_model.py:11-44
  ResidualMLP                 :336-403
  CausalMultiChannelConvBlock :128-212     MultiChannelConvBlock :214-253
  TargetEncoder :406-575  SourceEncoder :589-721  ConditionalEncoder :743-820
  Decoder :823-979  SeqVaeTeb :982-1192 (forward :1084-1131, loss :1133-1192)
  step: ref/model/graph_model.py:700-726 (zero_grad, fwd, loss, bwd, clip, AdamW)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def geometric(a, b, n):
    r = (b / a) ** (1 / (n + 1))
    out, cur = [], r
    for _ in range(n):
        out.append(int(round(a * cur)))
        cur *= r
    return tuple(out + [b])


class ResMLP(nn.Module):
    def __init__(self, din, dims, final_act=True, act="relu", skip=True):
        super().__init__()
        self.input_norm = nn.LayerNorm(din)
        mods, d = [], din
        for i, h in enumerate(dims):
            last = i == len(dims) - 1
            mods.append(nn.Linear(d, h))
            if not (last and not final_act):
                mods.append(nn.LayerNorm(h))
            if not last:
                mods.append(nn.GELU() if act == "gelu" else nn.ReLU())
            d = h
        self.body = nn.Sequential(*mods)
        self.final_act = final_act
        self.act = act
        self.skip = skip
        if skip:
            self.skip_proj = nn.Linear(din, dims[-1]) if din != dims[-1] else nn.Identity()

    def forward(self, x):
        x0 = self.input_norm(x)
        y = self.body(x0)
        if self.final_act:
            y = F.gelu(y) if self.act == "gelu" else F.relu(y)
        return y + self.skip_proj(x0) if self.skip else y


class CausalBlock(nn.Module):
    def __init__(self, c, k):
        super().__init__()
        self.k = k
        self.conv = nn.Conv1d(c, c, k, bias=False)
        self.bn_layer = nn.BatchNorm1d(c, momentum=0.9)

    def forward(self, x):
        return F.relu(self.bn_layer(self.conv(F.pad(x, (self.k - 1, 0)))))


class ReflBlock(nn.Module):
    def __init__(self, cin, cout, k, up=False, tanh=False):
        super().__init__()
        self.p, self.up, self.tanh = (k - 1) // 2, up, tanh
        self.conv = nn.Conv1d(cin, cout, k, bias=False)
        self.bn_layer = nn.BatchNorm1d(cout, momentum=0.9)

    def forward(self, x):
        if self.up:
            x = F.interpolate(x, scale_factor=2, mode="linear", align_corners=False)
        p = self.p
        if p > 0:
            if x.shape[-1] <= p:
                x = F.pad(x, (p, p), mode="replicate")
            else:
                x = torch.cat([x[..., 1:p + 1].flip(-1), x, x[..., -p - 1:-1].flip(-1)], -1)
        y = self.bn_layer(self.conv(x))
        return torch.tanh(y) if self.tanh else F.relu(y)


def _wrap(m):
    s = nn.Sequential(); s.add_module("0", m); return s


class SourceEnc(nn.Module):
    def __init__(self, cin=130):
        super().__init__()
        self.mlp = ResMLP(cin, geometric(130, 32, 5), final_act=False)
        self.conv = nn.Sequential(*[CausalBlock(32, k) for k in (3, 5, 7)])
        self.fused_norm = nn.LayerNorm(32)
        self.lstm_norm = nn.LayerNorm(64)
        self.lstm = nn.LSTM(32, 64, 4, batch_first=True)
        self.pre_output = ResMLP(64, geometric(64, 32, 4), final_act=True)
        self.mu_layer = ResMLP(32, geometric(32, 32, 4), final_act=False)

    def forward(self, x):
        h = self.conv(self.mlp(x).transpose(1, 2)).transpose(1, 2)
        h, _ = self.lstm(self.fused_norm(h))
        return self.mu_layer(self.pre_output(self.lstm_norm(h)))


class TargetEnc(nn.Module):
    def __init__(self, c_st=43, c_ph=44):
        super().__init__()
        self.mlp_scattering = _wrap(ResMLP(c_st, geometric(43, 16, 4), final_act=False, act="gelu"))
        self.mlp_phase = ResMLP(c_ph, geometric(44, 16, 4), final_act=False)
        self.conv_scattering = nn.Sequential(*[CausalBlock(16, k) for k in (3, 5, 7)])
        self.conv_phase = nn.Sequential(*[CausalBlock(16, k) for k in (3, 5, 7)])
        self.scatter_fused_norm = nn.LayerNorm(16)
        self.phase_fused_norm = nn.LayerNorm(16)
        self.lstm_norm = nn.LayerNorm(64)
        self.cross_modal_fusion = ResMLP(32, geometric(32, 20, 5), final_act=False)
        self.lstm = nn.LSTM(20, 64, 4, batch_first=True)
        self.pre_output = ResMLP(64, geometric(64, 32, 5), final_act=True)
        self.mu_layer = ResMLP(32, geometric(32, 32, 32), final_act=False)
        self.logvar_layer = ResMLP(32, geometric(32, 64, 4), final_act=False)

    def forward(self, ys, yp):
        a = self.scatter_fused_norm(self.conv_scattering(self.mlp_scattering(ys).transpose(1, 2)).transpose(1, 2))
        b = self.phase_fused_norm(self.conv_phase(self.mlp_phase(yp).transpose(1, 2)).transpose(1, 2))
        h, _ = self.lstm(self.cross_modal_fusion(torch.cat([a, b], -1)))
        h = self.pre_output(self.lstm_norm(h))
        return self.mu_layer(h), torch.clamp(self.logvar_layer(h), -10, 10)


class CondEnc(nn.Module):
    def __init__(self):
        super().__init__()
        hd = geometric(64, 32, 8)
        self.mlp = ResMLP(64, hd[:5], final_act=True)
        self.fc_mu = ResMLP(hd[4], hd[5:], final_act=False, skip=False)
        self.fc_logvar = ResMLP(hd[4], hd[5:], final_act=False, skip=False)

    def forward(self, hx, hy):
        h = self.mlp(torch.cat([hx, hy], -1))
        return self.fc_mu(h), self.fc_logvar(h)


class Dec(nn.Module):
    def __init__(self, R):
        super().__init__()
        self.linear = nn.Sequential(ResMLP(32, geometric(32, 50, 5)), ResMLP(50, geometric(50, 87, 5)))
        spec = [(87, 77, 11, 0), (77, 66, 9, 1), (66, 55, 7, 1), (55, 44, 5, 0),
                (44, 33, 5, 1), (33, 22, 3, 1), (22, 11, 3, 0), (11, 1, 3, 0)]
        self.conv = nn.Sequential(*[ReflBlock(a, b, k, bool(u)) for a, b, k, u in spec])
        self.output_mu = ResMLP(R, (R, R), final_act=False, skip=False)
        self.output_logvar = ResMLP(R, (R, R), final_act=False, skip=False)

    def forward(self, z):
        lin = self.linear(z)
        h = self.conv(lin.transpose(1, 2)).flatten(1)
        return lin, self.output_mu(h), self.output_logvar(h)


def kld(mp, lp, mq, lq):
    return (0.5 * (lp - lq - 1 + (lq.exp() + (mq - mp) ** 2) / lp.exp())).sum(-1).mean()


class SeqVaeTebRef(nn.Module):
    """Encoder input widths are parameters (the reference hard-codes 43 / 44 / 130 at
    ref/model/vae_teb_model.py:429,438,613; the hidden schedules keep those anchors, as
    the HIP model does), so the literal J=6 Q=1 front-end (8 / 13 / 7) has an oracle."""

    def __init__(self, sequence_length=300, scattering_channels=43, phase_channels=44, cross_phase_channels=130):
        super().__init__()
        self.source_encoder = SourceEnc(cross_phase_channels)
        self.target_encoder = TargetEnc(scattering_channels, phase_channels)
        self.conditional_encoder = CondEnc()
        self.decoder = Dec(16 * sequence_length)

    def forward(self, y_st, y_ph, x_ph, eps):
        mx = self.source_encoder(x_ph)
        my, lv = self.target_encoder(y_st, y_ph)
        lvp, c = torch.split(lv, 32, -1)
        mq, lq = self.conditional_encoder(mx, c)
        mq = mq + my
        z = mq + eps * torch.exp(0.5 * lq)
        lin, mu, lvr = self.decoder(z)
        return dict(z=z, linear_output=lin, mu_pr=mu, logvar_pr=lvr, mu_prior=my, logvar_prior=lvp,
                    mu_post=mq, logvar_post=lq)

    def measure_transfer_entropy(self, y_st, y_ph, x_ph, reduce_mean=False):
        """ref/model/vae_teb_model.py:1194-1226: eval mode (left set), no grad, KL(q || p)
        elementwise (B, S, 32) or the mean of its latent sums."""
        self.eval()
        with torch.no_grad():
            mx = self.source_encoder(x_ph)
            my, lv = self.target_encoder(y_st, y_ph)
            lvp, c = torch.split(lv, 32, -1)
            mq, lq = self.conditional_encoder(mx, c)
            mq = mq + my
            k = 0.5 * (lvp - lq - 1 + (lq.exp() + (mq - my) ** 2) / lvp.exp())
        return k.sum(-1).mean() if reduce_mean else k

    @staticmethod
    def compute_loss(fw, y_st, y_ph, y_raw, beta=1.0):
        lin = fw["linear_output"]
        mse = F.mse_loss(lin, torch.cat([y_st, y_ph], -1)) if (lin.shape[-1] == 87 and y_st.shape[-1] == 43
                                                                 and y_ph.shape[-1] == 44) else lin.new_zeros(())
        lv = fw["logvar_pr"]
        nll = (0.5 * (lv + (y_raw - fw["mu_pr"]) ** 2 / lv.exp())).mean()
        k = kld(fw["mu_prior"], fw["logvar_prior"], fw["mu_post"], fw["logvar_post"])
        return dict(mse_loss=mse, nll_loss=nll, kld_loss=k, reconstruction_loss=mse + nll,
                    total_loss=mse + nll + beta * k)


def train_step(model, batch, eps, beta, lr=1e-3, clip=1.0, betas=(0.9, 0.98), wd=1e-4):
    """One reference training step (graph_model.py:707-726, fp32 path)."""
    model.train()
    model.zero_grad(set_to_none=True)
    fw = model(batch["y_st"], batch["y_ph"], batch["x_ph"], eps)
    losses = model.compute_loss(fw, batch["y_st"], batch["y_ph"], batch["y_raw"], beta)
    losses["total_loss"].backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    gn = torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wd, eps=1e-8, betas=betas)
    opt.step()
    return fw, losses, grads, gn


class TinyVaeTebRef(nn.Module):
    """Config 1 from reference block semantics."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Sequential(_Causal1(1, 16, 3), _Causal1(16, 16, 5))
        self.mu = ResMLP(16, (8,), final_act=False)
        self.logvar = ResMLP(16, (8,), final_act=False)
        self.dec = nn.Sequential(ReflBlock(8, 16, 3), ReflBlock(16, 2, 3, tanh=True))

    def forward(self, x, eps):
        h = self.enc(x).transpose(1, 2)
        mu, lv = self.mu(h), self.logvar(h)
        out = self.dec((mu + eps * torch.exp(0.5 * lv)).transpose(1, 2))
        zero = torch.zeros_like(mu)
        kl = kld(zero, zero, mu, lv)
        nll = (0.5 * (out[:, 1] + (x[:, 0] - out[:, 0]) ** 2 / out[:, 1].exp())).mean()
        return dict(mu=mu, logvar=lv, mu_r=out[:, 0], lv_r=out[:, 1], kld=kl, nll=nll, total=nll + kl)


class _Causal1(CausalBlock):
    def __init__(self, cin, cout, k):
        nn.Module.__init__(self)
        self.k = k
        self.conv = nn.Conv1d(cin, cout, k, bias=False)
        self.bn_layer = nn.BatchNorm1d(cout, momentum=0.9)
