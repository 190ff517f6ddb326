"""sgan.models for MI355X: drop-in TrajectoryGenerator / TrajectoryDiscriminator.

Same classes, constructor keywords, forward() signatures and state-dict keys
as the reference's sgan/models.py (so scripts/train.py, scripts/evaluate_model.py
and reference checkpoints work unchanged), but the hot path runs on the
libsgg.so HIP kernels (sgan/kernels.py):

  - social pooling (PoolHiddenNet)        -> sgg_pool_fwd / sgg_pool_bwd
  - GAT attention + softmax + aggregate   -> sgg_gat_fwd / sgg_gat_bwd
  - GCN / GAT node transforms X W, Linear -> sgg_xw (fp32 MFMA)
  - group structure, R / R^T pooling       -> sgg_group_index, sgg_seg_reduce/gather

Scene bookkeeping is an int32 CSR built once per batch (sgan/scene.py)
instead of a `.item()` per scene per module.  The encoder LSTM and the 12-step
decoder rollout are single fused launches (sgg_lstm_fwd / sgg_lstm_bwd).

Checkpoint families: TrajectoryGenerator.load_state_dict reads the family off
the state's key set (family_of) and rebuilds the family's modules before the
(strict) load, so the reference's scripts/evaluate_model.py:30-52 loads every
family's g_state unchanged.

Extra keyword-only arguments beyond the reference's are optional and default
to the reference behaviour:
  TrajectoryGenerator(..., graph='gat'|'gcn'|'sgangat'|'vanilla')  selects
      the family up front, e.g. to train one from scratch ('gat' = the committed
      forward, models.py:903-905; 'gcn' = the sgan-g(-p) checkpoint families,
      :902; 'sgangat' = the sgangat-g-p family: the batched multi-head GAT of
      the commented sgan/GAT.py:6-106 text, then gcn_module; n_heads is then
      the per-layer head list, e.g. [4, 1]; 'vanilla' = upstream Social-GAN,
      the sgan-models / sgan-p-models families: mlp_decoder_context, the
      commented models.py:796-804 / :898, and no group module).
  forward(..., scenes=SceneIndex)  reuses a precomputed scene index.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .scene import SceneIndex

# ---------------------------------------------------------------------------
# batch bookkeeping
# ---------------------------------------------------------------------------
_SCENE_CACHE = {"sse": None, "ver": None, "dev": None, "idx": None}


def scene_index(seq_start_end, device):
    """SceneIndex of a batch, cached on the identity of the seq_start_end
    tensor (generator_step calls G best_k times with the same one).  The
    cache holds a reference to the tensor so its memory cannot be recycled
    into a different batch while cached."""
    c = _SCENE_CACHE
    if c["sse"] is seq_start_end and c["ver"] == seq_start_end._version and c["dev"] == device:
        return c["idx"]
    idx = SceneIndex.from_seq_start_end(seq_start_end, device)
    c.update(sse=seq_start_end, ver=seq_start_end._version, dev=device, idx=idx)
    return idx


def _scenes(seq_start_end, device, scenes):
    if scenes is not None:
        return scenes
    return scene_index(seq_start_end, device)


def make_mlp(dim_list, activation="relu", batch_norm=True, dropout=0):
    """Same layer layout as the reference (models.py:7-20) so state-dict keys
    (`.0.weight`, `.2.weight`, ...) match; executed by run_mlp."""
    layers = []
    for dim_in, dim_out in zip(dim_list[:-1], dim_list[1:]):
        layers.append(nn.Linear(dim_in, dim_out))
        if batch_norm:
            layers.append(nn.BatchNorm1d(dim_out))
        if activation == "relu":
            layers.append(nn.ReLU())
        elif activation == "leakyrelu":
            layers.append(nn.LeakyReLU())
        if dropout > 0:
            layers.append(nn.Dropout(p=dropout))
    return nn.Sequential(*layers)


def run_mlp(seq, x):
    """Run a make_mlp Sequential with every Linear on the MFMA node transform
    (ReLU fused into its epilogue)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Linear):
            fuse = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = K.linear(x, m, act=1 if fuse else 0)
            i += 2 if fuse else 1
            continue
        if isinstance(m, nn.BatchNorm1d):
            x = m(x)
        else:
            x = m(x)
        i += 1
    return x


def get_noise(shape, noise_type):
    """models.py:23-29: drawn from the HOST torch RNG (same stream as the
    reference, which draws on the CPU and copies)."""
    if noise_type == "gaussian":
        return torch.randn(*shape)
    if noise_type == "uniform":
        return torch.rand(*shape).sub_(0.5).mul_(2.0)
    raise ValueError('Unrecognized noise type "%s"' % noise_type)


# ---------------------------------------------------------------------------
# encoder / decoder (models.py:32-178) -> sgg_lstm_fwd / sgg_lstm_bwd
# ---------------------------------------------------------------------------
class Encoder(nn.Module):
    def __init__(self, embedding_dim=64, h_dim=64, mlp_dim=1024, num_layers=1, dropout=0.0):
        super().__init__()
        self.mlp_dim = 1024
        self.h_dim = h_dim
        self.embedding_dim = embedding_dim
        self.num_layers = num_layers
        self.spatial_embedding = nn.Linear(2, embedding_dim)
        self.encoder = nn.LSTM(embedding_dim, h_dim, num_layers, dropout=dropout)

    def forward(self, obs_traj, proj_u=None):
        """Fused sgg_lstm_fwd over all T steps; the Linear(2, E) embedding is
        folded into the input weights (A = W_ih We, b = W_ih be + b_ih + b_hh).
        proj_u = (Wu, cu): also return U = h Wu^T + cu (None where the kernel
        has no epilogue for these sizes) -- the pooling net's first layer."""
        if self.num_layers != 1:
            raise NotImplementedError("fused LSTM kernel: num_layers must be 1 (all reference configs)")
        if proj_u is not None:
            h, U = K.lstm_sequence(obs_traj, self.encoder, self.spatial_embedding, proj_u=proj_u)
            return h.unsqueeze(0), U
        h, _ = K.lstm_sequence(obs_traj, self.encoder, self.spatial_embedding)
        return h.unsqueeze(0)


class Decoder(nn.Module):
    def __init__(self, seq_len, embedding_dim=64, h_dim=128, mlp_dim=1024, num_layers=1,
                 pool_every_timestep=True, dropout=0.0, bottleneck_dim=1024, activation="relu",
                 batch_norm=True, pooling_type="pool_net", neighborhood_size=2.0, grid_size=8):
        super().__init__()
        self.seq_len = seq_len
        self.mlp_dim = mlp_dim
        self.h_dim = h_dim
        self.embedding_dim = embedding_dim
        self.pool_every_timestep = pool_every_timestep
        self.spatial_embedding = nn.Linear(2, embedding_dim)
        self.decoder = nn.LSTM(embedding_dim, h_dim, num_layers, dropout=dropout)
        self.hidden2pos = nn.Linear(h_dim, 2)
        if pool_every_timestep:
            if pooling_type == "pool_net":
                self.pool_net = PoolHiddenNet(embedding_dim=embedding_dim, h_dim=h_dim, mlp_dim=mlp_dim,
                                              bottleneck_dim=bottleneck_dim, activation=activation,
                                              batch_norm=batch_norm, dropout=dropout)
            self.mlp = make_mlp([h_dim + bottleneck_dim, mlp_dim, h_dim], activation=activation,
                                batch_norm=batch_norm, dropout=dropout)

    def forward(self, last_pos, last_pos_rel, state_tuple, seq_start_end, scenes=None):
        if not self.pool_every_timestep:
            # the whole 12-step rollout (LSTM step -> hidden2pos -> embedding
            # of the predicted displacement) is one sgg_lstm_fwd launch
            h0, c0 = state_tuple
            h, rel = K.lstm_sequence(last_pos_rel, self.decoder, self.spatial_embedding, h0=h0[0],
                                     c0=c0[0] if c0 is not None else None,
                                     proj=self.hidden2pos, decoder=True, T=self.seq_len)
            return rel, h.unsqueeze(0)
        B = last_pos.size(0)
        x = K.linear(last_pos_rel, self.spatial_embedding).view(1, B, self.embedding_dim)
        outs = []
        for _ in range(self.seq_len):
            y, state_tuple = self.decoder(x, state_tuple)
            rel = K.linear(y.view(-1, self.h_dim), self.hidden2pos)
            curr = rel + last_pos
            if self.pool_every_timestep:
                h = state_tuple[0]
                pool_h = self.pool_net(h, seq_start_end, curr, scenes=scenes)
                h = run_mlp(self.mlp, torch.cat([h.view(-1, self.h_dim), pool_h], dim=1))
                state_tuple = (h.unsqueeze(0), state_tuple[1])
            x = K.linear(rel, self.spatial_embedding).view(1, B, self.embedding_dim)
            outs.append(rel.view(B, -1))
            last_pos = curr
        return torch.stack(outs, dim=0), state_tuple[0]


# ---------------------------------------------------------------------------
# social pooling (models.py:458-549) -> sgg_pool_*
# ---------------------------------------------------------------------------
class PoolHiddenNet(nn.Module):
    """Pooling module as proposed in Social-GAN.  The pair MLP runs fused in
    sgg_pool_fwd; the spatial embedding is folded into the first layer
    (A = W1e We, c = W1e be + b1, sgg_fold_fwd) inside the autograd op, which
    returns the raw parameters' gradients."""

    def __init__(self, embedding_dim=64, h_dim=64, mlp_dim=1024, bottleneck_dim=1024, activation="relu",
                 batch_norm=True, dropout=0.0):
        super().__init__()
        self.mlp_dim = 1024
        self.h_dim = h_dim
        self.bottleneck_dim = bottleneck_dim
        self.embedding_dim = embedding_dim
        self.activation, self.batch_norm, self.dropout = activation, batch_norm, dropout
        self.spatial_embedding = nn.Linear(2, embedding_dim)
        self.mlp_pre_pool = make_mlp([embedding_dim + h_dim, 512, bottleneck_dim], activation=activation,
                                     batch_norm=batch_norm, dropout=dropout)

    def fused_ok(self):
        return not (self.batch_norm or self.activation != "relu" or self.dropout > 0)

    def forward(self, h_states, seq_start_end, end_pos, scenes=None, link=None, U=None):
        """U (optional): h W1[:, E:]^T + c already computed by the encoder
        kernel's epilogue (K.pool_u_spec)."""
        if not self.fused_ok():
            raise NotImplementedError("the fused pooling kernel implements the reference configs "
                                      "(batch_norm=0, relu, dropout=0)")
        sc = _scenes(seq_start_end, end_pos.device, scenes)
        l1, l2 = self.mlp_pre_pool[0], self.mlp_pre_pool[2]
        emb = self.spatial_embedding
        return K.social_pool(h_states.reshape(-1, self.h_dim), end_pos, l1.weight, emb.weight, emb.bias, l1.bias,
                             l2.weight, l2.bias, sc, link=link, U=U)


# ---------------------------------------------------------------------------
# GAT (models.py:184-294) -> sgg_xw + sgg_gat_*
# ---------------------------------------------------------------------------
class GraphAttentionLayer(nn.Module):
    def __init__(self, in_features, out_features, dropout, alpha, concat=True):
        super().__init__()
        self.dropout = dropout
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = alpha
        self.concat = concat
        self.W = nn.Parameter(torch.empty(size=(in_features, out_features)))
        nn.init.xavier_uniform_(self.W.data, gain=1.414)
        self.a = nn.Parameter(torch.empty(size=(2 * out_features, 1)))
        nn.init.xavier_uniform_(self.a.data, gain=1.414)

    def forward(self, h, graph, epilogue=None):
        """graph: kernels.SegmentGraph.  epilogue defaults to ELU when concat
        (models.py:207-210); GAT passes 2 to fuse its ELU + log_softmax."""
        if self.dropout > 0 and self.training:
            raise NotImplementedError("attention dropout is not implemented in the fused kernel (dropout1=0)")
        wh = K.xw(h, self.W)
        epi = (1 if self.concat else 0) if epilogue is None else epilogue
        return K.gat_attention(wh, self.a, self.alpha, graph, epi)


class GAT(nn.Module):
    def __init__(self, nfeat, nhid, nclass, dropout, alpha, nheads):
        super().__init__()
        self.dropout = dropout
        self.attentions = [GraphAttentionLayer(nfeat, nhid, dropout=dropout, alpha=alpha, concat=True)
                           for _ in range(nheads)]
        for i, attention in enumerate(self.attentions):
            self.add_module("attention_{}".format(i), attention)
        self.out_att = GraphAttentionLayer(nhid * nheads, nclass, dropout=dropout, alpha=alpha, concat=False)

    def forward(self, x, graph):
        """models.py:231-237: heads (ELU) concatenated -> out_att -> ELU ->
        log_softmax(dim=1); the last two fused into the kernel epilogue."""
        heads = [att(x, graph) for att in self.attentions]
        x = heads[0] if len(heads) == 1 else torch.cat(heads, dim=1)
        return self.out_att(x, graph, epilogue=2)


class GATEncoder(nn.Module):
    def __init__(self, n_units, n_heads, dropout, alpha):
        super().__init__()
        self.gat_intra = GAT(40, 72, 16, dropout, alpha, n_heads)
        self.gat_inter = GAT(16, 72, 16, dropout, alpha, n_heads)
        self.out_embedding = nn.Linear(16 * 2, 24)

    def fused_params(self):
        """The parameters in the order of the fused kernel's slab (sgg.h)."""
        ps = []
        for gat in (self.gat_intra, self.gat_inter):
            for att in gat.attentions:
                ps += [att.W, att.a]
            ps += [gat.out_att.W, gat.out_att.a]
        return ps + [self.out_embedding.weight, self.out_embedding.bias]

    def fused_ok(self, sc, need_grad):
        """The one-launch path (sgg_gatenc_*) takes these scenes."""
        return ((self.gat_intra.dropout == 0 or not self.training)
                and K.gat_encoder_fused_ok(sc, len(self.gat_intra.attentions), need_grad))

    def forward(self, h_states, seq_start_end, end_pos, end_group, scenes=None, link=None, companion=None):
        """h_states: (B, 40), or the pair (encoder state, pooled vector) whose
        concatenation it is (the fused kernel reads both blocks in place).
        link: GradLink shared with the pooling net (see kernels.GradLink).
        companion: a kernels.GatEncCompanion (a no-grad batch through the
        same module) run in the same launch; the fused path only."""
        x2 = None
        if isinstance(h_states, (tuple, list)):
            h_states, x2 = h_states
        sc = _scenes(seq_start_end, h_states.device, scenes)
        if sc.max_n > 128:
            raise ValueError("GAT kernels hold <= 128 peds per scene (got %d)" % sc.max_n)
        nh = len(self.gat_intra.attentions)
        params = self.fused_params()
        need_grad = torch.is_grad_enabled() and (h_states.requires_grad or (x2 is not None and x2.requires_grad)
                                                 or any(p.requires_grad for p in params))
        if self.fused_ok(sc, need_grad):
            # one launch per direction for the whole module (sgg_gatenc_fwd / _bwd)
            return K.gat_encoder(h_states, end_group, sc, nh, self.gat_intra.attentions[0].alpha, params, x2=x2,
                                 link=link, companion=companion)
        if companion is not None:
            raise ValueError("GATEncoder: a companion batch needs the one-launch path (fused_ok)")
        if x2 is not None:
            h_states = torch.cat([h_states, x2], dim=1)
        g = sc.groups(end_group.reshape(-1))
        intra_graph = K.SegmentGraph(sc.scene_off, sc.S, sc.max_n, 0, g.labels)
        inter_graph = K.SegmentGraph(g.group_off, sc.S, sc.max_n, 1, None)
        intra = self.gat_intra(h_states, intra_graph)                 # B x 16
        gin = K.group_mean(intra, g)                                   # R @ intra  (cap x 16)
        gout = self.gat_inter(gin, inter_graph)                        # cap x 16
        inter = K.group_unpool(gout, g, scale=True)                    # R^T @ gout (B x 16)
        return K.linear(torch.cat([intra, inter], dim=1), self.out_embedding)


# ---------------------------------------------------------------------------
# batched multi-head GAT of the sgangat checkpoint family (the commented-out
# BatchMultiHeadGraphAttention / GAT / GATEncoder text of sgan/GAT.py:6-106)
# -> sgg_seg_norm_* + sgg_xw + multi-head sgg_gat_*
# ---------------------------------------------------------------------------
class BatchMultiHeadGraphAttention(nn.Module):
    """GAT.py:6-55 text: per head h, h'_h = x w_h; e_ij = LeakyReLU_0.2(
    h'_i.a_src + h'_j.a_dst) over the complete scene graph (no adjacency);
    softmax over j; out_h = att h'_h + bias.  All heads in one kernel launch;
    the (n, heads*F_out) output is the transpose(1, 2).view concat of :86."""

    def __init__(self, n_head, f_in, f_out, attn_dropout, bias=True):
        super().__init__()
        self.n_head, self.f_in, self.f_out = n_head, f_in, f_out
        self.w = nn.Parameter(torch.Tensor(n_head, f_in, f_out))
        self.a_src = nn.Parameter(torch.Tensor(n_head, f_out, 1))
        self.a_dst = nn.Parameter(torch.Tensor(n_head, f_out, 1))
        self.leaky_relu = nn.LeakyReLU(negative_slope=0.2)
        self.softmax = nn.Softmax(dim=-1)
        self.dropout = nn.Dropout(attn_dropout)
        if bias:
            self.bias = nn.Parameter(torch.Tensor(f_out))
            nn.init.constant_(self.bias, 0)
        else:
            self.register_parameter("bias", None)
        nn.init.xavier_uniform_(self.w, gain=1.414)
        nn.init.xavier_uniform_(self.a_src, gain=1.414)
        nn.init.xavier_uniform_(self.a_dst, gain=1.414)

    def forward(self, x, graph, epilogue):
        if self.dropout.p > 0 and self.training:
            raise NotImplementedError("attention dropout is not implemented in the fused kernel (dropout1=0)")
        H, Fi, Fo = self.n_head, self.f_in, self.f_out
        w_all = self.w.permute(1, 0, 2).reshape(Fi, H * Fo)                 # [w_0 | .. | w_{H-1}]
        wh = K.xw(x, w_all)                                                  # n x H*Fo
        return K.gat_attention_ex(wh, self.a_src, self.a_dst, 0.2, graph, epilogue, heads=H, bias=self.bias)

    def __repr__(self):
        return "%s (%d -> %d -> %d)" % (self.__class__.__name__, self.n_head, self.f_in, self.f_out)


class BatchGAT(nn.Module):
    """GAT.py:58-89 text: per layer InstanceNorm1d over the scene's peds, the
    multi-head attention, then ELU (all but the last layer, whose single head
    is squeezed).  The reference's norm_list modules hold no parameters."""

    def __init__(self, n_units, n_heads, dropout=0.2, alpha=0.2):
        super().__init__()
        self.n_layer = len(n_units) - 1
        self.dropout = dropout
        self.layer_stack = nn.ModuleList()
        for i in range(self.n_layer):
            f_in = n_units[i] * n_heads[i - 1] if i else n_units[i]
            self.layer_stack.append(BatchMultiHeadGraphAttention(n_heads[i], f_in=f_in, f_out=n_units[i + 1],
                                                                 attn_dropout=dropout))
        if n_heads[self.n_layer - 1] != 1:
            raise ValueError("the last batched GAT layer must have one head (GAT.py:83 squeezes it)")

    def forward(self, x, graph):
        """x: (n, n_units[0]) or its two column blocks (h, pool_h).  Each layer
        is one sgg_gat_layer_fwd launch (norm + node transform + attention)
        when it fits the kernel (LAYER_FUSED), else the per-op path."""
        if self.dropout > 0 and self.training:
            raise NotImplementedError("dropout between GAT layers is not implemented (dropout1=0)")
        for i, layer in enumerate(self.layer_stack):
            epi = 0 if i + 1 == self.n_layer else 1                          # ELU fused into the kernel
            if BatchGAT.LAYER_FUSED and K.gat_layer_ok(layer.f_in, layer.f_out, layer.n_head, graph.max_seg, epi):
                x = K.gat_layer(x, layer.w, layer.a_src, layer.a_dst, layer.bias, graph, epi)
                continue
            if isinstance(x, tuple):
                x = torch.cat(x, dim=1)
            x = K.seg_instance_norm(x, graph.seg_off, graph.nseg)
            x = layer(x, graph, epi)
        return x

    def forward_pair(self, xa, graph_a, xb, graph_b):
        """forward() of two batches, a without autograd (the discriminator
        step's) and b (the generator step's): layer by layer, each fused
        layer of both batches in ONE launch (kernels.gat_layer_pair,
        sgg_gat_layer_fwd2); each result as forward() computes it."""
        if self.dropout > 0 and self.training:
            raise NotImplementedError("dropout between GAT layers is not implemented (dropout1=0)")
        for i, layer in enumerate(self.layer_stack):
            epi = 0 if i + 1 == self.n_layer else 1
            ok = BatchGAT.LAYER_FUSED and all(K.gat_layer_ok(layer.f_in, layer.f_out, layer.n_head, g.max_seg, epi)
                                              for g in (graph_a, graph_b))
            if ok:
                with K.gat_layer_pair():
                    with torch.no_grad():
                        xa = K.gat_layer(xa, layer.w, layer.a_src, layer.a_dst, layer.bias, graph_a, epi)
                    xb = K.gat_layer(xb, layer.w, layer.a_src, layer.a_dst, layer.bias, graph_b, epi)
                continue
            with torch.no_grad():
                xa = layer(K.seg_instance_norm(torch.cat(xa, 1) if isinstance(xa, tuple) else xa, graph_a.seg_off,
                                               graph_a.nseg), graph_a, epi)
            xb = layer(K.seg_instance_norm(torch.cat(xb, 1) if isinstance(xb, tuple) else xb, graph_b.seg_off,
                                           graph_b.nseg), graph_b, epi)
        return xa, xb

    LAYER_FUSED = True


class BatchGATEncoder(nn.Module):
    """GAT.py:92-106 text: the batched GAT run over each scene's peds
    (complete graph); (B, n_units[0]) -> (B, n_units[-1])."""

    def __init__(self, n_units, n_heads, dropout, alpha):
        super().__init__()
        self.gat_net = BatchGAT(n_units, n_heads, dropout, alpha)

    def forward(self, h_states, seq_start_end, scenes=None):
        """h_states: (B, n_units[0]) or its two column blocks (h, pool_h)."""
        dev = (h_states[0] if isinstance(h_states, tuple) else h_states).device
        sc = _scenes(seq_start_end, dev, scenes)
        if sc.max_n > 128:
            raise ValueError("GAT kernels hold <= 128 peds per scene (got %d)" % sc.max_n)
        return self.gat_net(h_states, K.SegmentGraph(sc.scene_off, sc.S, sc.max_n, 1, None))

    def forward_pair(self, ha, sca, hb, scb):
        """forward() of two batches (a without autograd) with each fused layer
        in one launch for both (BatchGAT.forward_pair)."""
        for sc in (sca, scb):
            if sc.max_n > 128:
                raise ValueError("GAT kernels hold <= 128 peds per scene (got %d)" % sc.max_n)
        return self.gat_net.forward_pair(ha, K.SegmentGraph(sca.scene_off, sca.S, sca.max_n, 1, None),
                                         hb, K.SegmentGraph(scb.scene_off, scb.S, scb.max_n, 1, None))


# ---------------------------------------------------------------------------
# GCN (models.py:552-712) -> sgg_seg_* + sgg_xw (ReLU fused)
# ---------------------------------------------------------------------------
class GCN(nn.Module):
    def __init__(self, input_dim=48, hidden_dim=72, out_dim=8, gcn_layers=2):
        super().__init__()
        self.X_dim = input_dim
        self.hidden_dim = hidden_dim
        self.out_dim = out_dim
        self.gcn_layers = gcn_layers
        self.W = torch.nn.ParameterList()
        for i in range(self.gcn_layers):
            if i == 0:
                self.W.append(nn.Parameter(torch.randn(self.X_dim, self.hidden_dim)))
            elif i == self.gcn_layers - 1:
                self.W.append(nn.Parameter(torch.randn(self.hidden_dim, self.out_dim)))
            else:
                self.W.append(nn.Parameter(torch.randn(self.hidden_dim, self.hidden_dim)))

    def forward(self, aggregate, X):
        """H <- ReLU((A H) W_l); `aggregate` applies the row-normalised A."""
        H = X
        for w in self.W:
            H = K.xw(aggregate(H), w, act=1)
        return H


class GCNModule(nn.Module):
    def __init__(self, input_dim=40, hidden_dim=72, out_dim=16, gcn_layers=2, final_dim=24):
        super().__init__()
        self.gcn_intra = GCN(input_dim=input_dim, hidden_dim=hidden_dim, out_dim=out_dim, gcn_layers=gcn_layers)
        self.gcn_inter = GCN(input_dim=16, hidden_dim=hidden_dim, out_dim=out_dim, gcn_layers=gcn_layers)
        self.out_embedding = nn.Linear(out_dim * 2, final_dim)

    def fused_params(self):
        """[W0, W1 of gcn_intra, W0, W1 of gcn_inter, out_embedding weight,
        bias] when the module has the shapes of the fused kernel (two layers,
        hidden 72, out 16: GCNModule's construction in TrajectoryGenerator),
        else None."""
        gi, gg = self.gcn_intra.W, self.gcn_inter.W
        if len(gi) != 2 or len(gg) != 2 or self.out_embedding.in_features != 32:
            return None
        if (gi[0].shape[1], tuple(gi[1].shape), tuple(gg[0].shape), tuple(gg[1].shape)) != (72, (72, 16), (16, 72),
                                                                                          (72, 16)):
            return None
        return [gi[0], gi[1], gg[0], gg[1], self.out_embedding.weight, self.out_embedding.bias]

    def fused_ok(self, sc, fin):
        """The one-launch path (sgg_gcnmod_*) takes these scenes and inputs."""
        params = self.fused_params()
        return (params is not None and params[0].shape[0] == fin
                and K.gcn_module_fused_ok(sc, fin, self.out_embedding.out_features))

    def forward(self, h_states, seq_start_end, end_pos, end_group, scenes=None, link=None, companion=None):
        """h_states: (B, 40), or the pair (encoder state, pooled vector) whose
        concatenation it is (the fused kernel reads both blocks in place).
        link: GradLink shared with the pooling net (see kernels.GradLink).
        companion: a kernels.GcnModCompanion run in the same launch (fused path)."""
        x2 = None
        if isinstance(h_states, (tuple, list)):
            h_states, x2 = h_states
        sc = _scenes(seq_start_end, h_states.device, scenes)
        params = self.fused_params()
        fin = h_states.shape[1] + (x2.shape[1] if x2 is not None else 0)
        if self.fused_ok(sc, fin):
            # one launch per direction for the whole module (sgg_gcnmod_fwd / _bwd)
            return K.gcn_module(h_states, end_group, sc, params, x2=x2, link=link, companion=companion)
        if companion is not None:
            raise ValueError("GCNModule: a companion batch needs the one-launch path (fused_ok)")
        if x2 is not None:
            h_states = torch.cat([h_states, x2], dim=1)
        g = sc.groups(end_group.reshape(-1))
        # A_intra = D^-1 M: row i averages its group (models.py:658-665)
        intra = self.gcn_intra(lambda H: K.group_unpool(K.group_mean(H, g), g, scale=False), h_states)
        gin = K.group_mean(intra, g)                                           # R @ intra
        gout = self.gcn_inter(lambda H: K.scene_mean_over_groups(H, g), gin)   # A_inter = 1/M
        inter = K.group_unpool(gout, g, scale=True)                            # R^T @ gout
        return K.linear(torch.cat([intra, inter], dim=1), self.out_embedding)


# ---------------------------------------------------------------------------
# generator / discriminator
# ---------------------------------------------------------------------------
class TrajectoryGenerator(nn.Module):
    def __init__(self, obs_len, pred_len, embedding_dim=64, encoder_h_dim=64, decoder_h_dim=128,
                 mlp_dim=1024, num_layers=1, noise_dim=(0,), noise_type="gaussian", noise_mix_type="ped",
                 pooling_type=None, pool_every_timestep=True, dropout=0.0, bottleneck_dim=1024,
                 activation="relu", batch_norm=True, neighborhood_size=2.0, grid_size=8,
                 n_units=[32, 16, 32], n_heads=4, dropout1=0, alpha=0.2, *, graph="gat"):
        super().__init__()
        if pooling_type and pooling_type.lower() == "none":
            pooling_type = None
        self.obs_len = obs_len
        self.pred_len = pred_len
        self.mlp_dim = mlp_dim
        self.encoder_h_dim = encoder_h_dim
        self.decoder_h_dim = decoder_h_dim
        self.embedding_dim = embedding_dim
        self.noise_dim = noise_dim
        self.num_layers = num_layers
        self.noise_type = noise_type
        self.noise_mix_type = noise_mix_type
        self.pooling_type = pooling_type
        self.noise_first_dim = 0
        self.pool_every_timestep = pool_every_timestep
        self.bottleneck_dim = 1024

        self.encoder = Encoder(embedding_dim=embedding_dim, h_dim=encoder_h_dim, mlp_dim=mlp_dim,
                               num_layers=num_layers, dropout=dropout)
        self.decoder = Decoder(pred_len, embedding_dim=embedding_dim, h_dim=decoder_h_dim, mlp_dim=mlp_dim,
                               num_layers=num_layers, pool_every_timestep=pool_every_timestep, dropout=dropout,
                               bottleneck_dim=bottleneck_dim, activation=activation, batch_norm=batch_norm,
                               pooling_type=pooling_type, grid_size=grid_size,
                               neighborhood_size=neighborhood_size)
        if pooling_type == "pool_net":
            self.pool_net = PoolHiddenNet(embedding_dim=self.embedding_dim, h_dim=encoder_h_dim, mlp_dim=mlp_dim,
                                          bottleneck_dim=bottleneck_dim, activation=activation,
                                          batch_norm=batch_norm)
        if self.noise_dim is None:
            self.noise_dim = None
        elif self.noise_dim[0] == 0:
            self.noise_dim = None
        else:
            self.noise_first_dim = noise_dim[0]
        self._family_args = dict(n_units=list(n_units), n_heads=n_heads, dropout1=dropout1, alpha=alpha,
                                 input_dim=encoder_h_dim + bottleneck_dim if pooling_type else encoder_h_dim,
                                 mlp_dim=mlp_dim, decoder_h_dim=decoder_h_dim, activation=activation,
                                 batch_norm=batch_norm, dropout=dropout)
        self._build_family(graph)

    # module set (and registration order, which fixes the optimizer-state
    # order) of each checkpoint family:
    #   gat     : committed models.py:800-812 -> gatencoder, gcn_module
    #   gcn     : sgan-g(-p)-models            -> mlp_decoder_context, gcn_module
    #   sgangat : sgangat-g-p-models           -> gatencoder.gat_net, mlp_decoder_context, gcn_module
    #   vanilla : sgan-models / sgan-p-models  -> mlp_decoder_context only (upstream Social-GAN,
    #             the commented models.py:796-804 / :898; no group module at all)
    # (mlp_decoder_context is carried by the gcn / sgangat checkpoints but not called)
    _FAMILY_MODULES = ("gatencoder", "mlp_decoder_context", "gcn_module")

    @staticmethod
    def family_of(keys):
        """The checkpoint family a generator state dict belongs to, from its
        key set alone (scripts/evaluate_model.py:30-52 builds the generator
        from the checkpoint's args, which name no family, then strict-loads
        g_state):  gatencoder.gat_net.* -> sgangat; gatencoder.gat_intra.* ->
        gat; gcn_module.* without a gatencoder -> gcn; neither -> vanilla."""
        keys = list(keys)
        if any(k.startswith("gatencoder.gat_net.") for k in keys):
            return "sgangat"
        if any(k.startswith("gatencoder.gat_intra.") for k in keys):
            return "gat"
        if any(k.startswith("gcn_module.") for k in keys):
            return "gcn"
        return "vanilla"

    def _build_family(self, graph, sgat_shapes=None):
        """(Re)build the family's modules.  Modules the old and new family
        share keep their objects (so e.g. gcn_module's parameters survive a
        gat -> gcn switch); the rest are created fresh and registered in the
        family's order.  sgat_shapes: [(heads, f_in, f_out)] per batched GAT
        layer, read from a state dict (the checkpoint's n_units / heads)."""
        if graph not in ("gat", "gcn", "sgangat", "vanilla"):
            raise ValueError("graph must be 'gat', 'gcn', 'sgangat' or 'vanilla'")
        a = self._family_args
        old = {n: self._modules.pop(n) for n in self._FAMILY_MODULES if n in self._modules}
        self.graph = graph
        ctx_out = a["decoder_h_dim"] - self.noise_first_dim
        if graph == "gat":
            ge = old.get("gatencoder")
            self.gatencoder = ge if isinstance(ge, GATEncoder) else GATEncoder(
                n_units=a["n_units"], n_heads=a["n_heads"], dropout=a["dropout1"], alpha=a["alpha"])
        elif graph == "sgangat":
            if sgat_shapes is not None:
                units = [sgat_shapes[0][1]] + [s[2] for s in sgat_shapes]
                heads = [s[0] for s in sgat_shapes]
            else:
                units = list(a["n_units"])
                nh = a["n_heads"]
                heads = list(nh) if isinstance(nh, (list, tuple)) else [nh] * (len(units) - 2) + [1]
            ge = old.get("gatencoder")
            same = (isinstance(ge, BatchGATEncoder)
                    and [(l.n_head, l.f_in, l.f_out) for l in ge.gat_net.layer_stack]
                    == [(h, (units[i] * heads[i - 1] if i else units[i]), units[i + 1]) for i, h in enumerate(heads)])
            self.gatencoder = ge if same else BatchGATEncoder(n_units=units, n_heads=heads, dropout=a["dropout1"],
                                                               alpha=a["alpha"])
        if graph in ("gcn", "sgangat") or (graph == "vanilla" and self.mlp_decoder_needed()):
            m = old.get("mlp_decoder_context")
            self.mlp_decoder_context = m if m is not None else make_mlp(
                [a["input_dim"], a["mlp_dim"], ctx_out], activation=a["activation"], batch_norm=a["batch_norm"],
                dropout=a["dropout"])
        if graph != "vanilla":
            m = old.get("gcn_module")
            self.gcn_module = m if m is not None else GCNModule(
                input_dim=a["input_dim"], hidden_dim=72, out_dim=16, gcn_layers=2, final_dim=ctx_out)
        # new modules follow the rest of the generator's device / dtype
        p0 = next(self.encoder.parameters())
        for n in self._FAMILY_MODULES:
            if n in self._modules and n not in old:
                self._modules[n].to(device=p0.device, dtype=p0.dtype)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        """nn.Module.load_state_dict after switching to the state's checkpoint
        family (family_of), so the reference's unchanged
        scripts/evaluate_model.py:30-52 -- TrajectoryGenerator(**checkpoint
        args), then a strict load of g_state -- works for every family
        (sgan-models / sgan-p-models, sgan-g(-p), sgan-gat, sgangat-g-p).  A
        state without any family module (a partial, strict=False load) keeps
        the current family."""
        keys = list(state_dict.keys())
        if strict or any(k.split(".")[0] in self._FAMILY_MODULES for k in keys):
            fam = self.family_of(keys)
            shapes = None
            if fam == "sgangat":
                ws = sorted((int(k.split(".")[3]), state_dict[k].shape) for k in keys
                            if k.startswith("gatencoder.gat_net.layer_stack.") and k.endswith(".w"))
                shapes = [tuple(int(d) for d in s) for _, s in ws]
            cur = None
            if fam == "sgangat" and isinstance(getattr(self, "gatencoder", None), BatchGATEncoder):
                cur = [(l.n_head, l.f_in, l.f_out) for l in self.gatencoder.gat_net.layer_stack]
            if fam != self.graph or (fam == "sgangat" and cur != shapes):
                self._build_family(fam, sgat_shapes=shapes)
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def add_noise(self, _input, seq_start_end, user_noise=None, scenes=None):
        """models.py:814-850 (noise drawn on the host, one draw per call)."""
        if not self.noise_dim:
            return _input
        sc = _scenes(seq_start_end, _input.device, scenes)
        if self.noise_mix_type == "global":
            noise_shape = (sc.S,) + tuple(self.noise_dim)
        else:
            noise_shape = (_input.size(0),) + tuple(self.noise_dim)
        z = user_noise if user_noise is not None else get_noise(noise_shape, self.noise_type)
        z = z.to(_input.device, non_blocking=True)
        if self.noise_mix_type == "global":
            z = z.index_select(0, sc.ped_scene_long())
        return torch.cat([_input, z], dim=1)

    def mlp_decoder_needed(self):
        return bool(self.noise_dim or self.pooling_type or self.encoder_h_dim != self.decoder_h_dim)

    def forward(self, obs_traj, obs_traj_rel, seq_start_end, obs_traj_g, user_noise=None, *, scenes=None):
        sc = _scenes(seq_start_end, obs_traj.device, scenes)
        noise_input = self.context(obs_traj, obs_traj_rel, seq_start_end, obs_traj_g, scenes=sc)
        return self.decode(noise_input, obs_traj, obs_traj_rel, seq_start_end, user_noise=user_noise, scenes=sc)

    def fold_specs(self):
        """The generator's input-embedding folds (encoder, pooling, decoder),
        computed together in one launch (kernels.prefold)."""
        specs = [K.lstm_fold_spec(self.encoder.encoder, self.encoder.spatial_embedding)]
        if self.pooling_type:
            specs.append(K.pool_fold_spec(self.pool_net))
        if not self.pool_every_timestep and self.num_layers == 1:
            specs.append(K.lstm_fold_spec(self.decoder.decoder, self.decoder.spatial_embedding))
        return specs

    def context(self, obs_traj, obs_traj_rel, seq_start_end, obs_traj_g, *, scenes=None):
        """The noise-independent part of forward() (models.py:877-906):
        encoder -> pooling -> GAT / GCN -> the decoder context (B, dec_h - noise).
        best-of-k sampling (scripts/train.py:443-455, evaluate_model.py:85)
        draws k samples that differ only in the noise appended after this
        point, so it runs once per batch and `decode(copies=k)` rolls the k
        samples out (the reference recomputes it k times, bit-identically)."""
        sc = _scenes(seq_start_end, obs_traj.device, scenes)
        if self.num_layers == 1:
            K.prefold(self.fold_specs())
        U = None
        if self.pooling_type == "pool_net" and self.num_layers == 1 and self.pool_net.fused_ok():
            # the pooling net's first layer (h half) in the encoder kernel's epilogue
            final_encoder_h, U = self.encoder(obs_traj_rel, proj_u=K.pool_u_spec(self.pool_net))
        else:
            final_encoder_h = self.encoder(obs_traj_rel)
        ctx = final_encoder_h.view(-1, self.encoder_h_dim)
        end_pos = obs_traj[-1]
        if self.pooling_type:
            two_block = self.graph in ("gat", "gcn") and self.mlp_decoder_needed()
            # the GAT encoder's / GCN module's gradient of h reaches the pooling
            # backward, which adds it in its own launch
            link = K.GradLink() if two_block and torch.is_grad_enabled() else None
            pool_h = self.pool_net(final_encoder_h, seq_start_end, end_pos, scenes=sc, link=link, U=U)
            if two_block:
                # the graph module reads [h | pool_h] as two blocks (no cat)
                module = self.gatencoder if self.graph == "gat" else self.gcn_module
                return module((ctx, pool_h), seq_start_end, end_pos, obs_traj_g[-1], scenes=sc, link=link)
            # (the batched GAT's first layer reads [h | pool_h] as two blocks)
            ctx = (ctx, pool_h) if self.graph == "sgangat" and self.mlp_decoder_needed() else torch.cat(
                [ctx, pool_h], dim=1)
        if self.mlp_decoder_needed():
            if self.graph == "gat":
                noise_input = self.gatencoder(ctx, seq_start_end, end_pos, obs_traj_g[-1], scenes=sc)
            elif self.graph == "vanilla":
                # upstream Social-GAN: noise_input = mlp_decoder_context(ctx) (models.py:898, dims
                # :796-804); both Linear layers on the MFMA node transform, ReLU fused
                noise_input = run_mlp(self.mlp_decoder_context, ctx)
            else:
                if self.graph == "sgangat":
                    ctx = self.gatencoder(ctx, seq_start_end, scenes=sc)
                noise_input = self.gcn_module(ctx, seq_start_end, end_pos, obs_traj_g[-1], scenes=sc)
        else:
            noise_input = ctx
        return noise_input

    def pair_ok(self, sc_a, sc_b):
        """context_pair runs its two batches' graph module (GATEncoder or
        GCNModule, two-block input; sgangat: the GCNModule after each batch's
        batched GAT) in one launch."""
        if not (self.graph in ("gat", "gcn", "sgangat") and self.pooling_type == "pool_net" and self.num_layers == 1
                and self.mlp_decoder_needed() and self.pool_net.fused_ok()):
            return False
        if self.graph == "gat":
            return self.gatencoder.fused_ok(sc_a, False) and self.gatencoder.fused_ok(sc_b, True)
        if self.graph == "sgangat":   # the GCNModule reads the batched GAT's output
            ps = self.gcn_module.fused_params()
            if ps is None:
                return False
            fin = ps[0].shape[0]
        else:
            fin = self.encoder_h_dim + self.pool_net.bottleneck_dim
        return self.gcn_module.fused_ok(sc_a, fin) and self.gcn_module.fused_ok(sc_b, fin)

    def context_pair(self, a, b):
        """context() of two batches: a = (obs_traj, obs_traj_rel, seq_start_end,
        obs_traj_g, scenes) without autograd -- the discriminator step's
        generator forward (scripts/train.py:400) -- and b with autograd -- the
        generator step's (:443-455).  G's weights do not change between the
        two steps (the discriminator step updates D only), so both contexts
        can be formed at the discriminator step: the encoders of both batches
        run in ONE launch (sgg_lstm_fwd_seg3, with the discriminator's
        observed-steps prefix when it is armed on a's input), so do the
        poolings (sgg_pool_fwd2) and the graph module (GATEncoder:
        sgg_gatenc_fwd2; GCNModule: sgg_gcnmod_fwd2), each result exactly as context() computes it.
        -> (context of a, context of b)."""
        obs_a, rel_a, sse_a, g_a, sc_a = a
        obs_b, rel_b, sse_b, g_b, sc_b = b
        if not self.pair_ok(sc_a, sc_b):
            with torch.no_grad():
                ca = self.context(obs_a, rel_a, sse_a, g_a, scenes=sc_a)
            return ca, self.context(obs_b, rel_b, sse_b, g_b, scenes=sc_b)
        K.prefold(self.fold_specs())
        u = K.pool_u_spec(self.pool_net)
        H = self.encoder_h_dim
        # both encoders (+ a discriminator prefix armed on a's input) in one
        # launch: a's is held until b's carries it (kernels.encoder_pair)
        with K.encoder_pair():
            with torch.no_grad():
                h_a, U_a = self.encoder(rel_a, proj_u=u)
            h_b, U_b = self.encoder(rel_b, proj_u=u)
        # (the two-block graph modules take the pooling's gradient link; the
        # batched GAT of sgangat reads [h | pool] through its own first layer)
        link = K.GradLink() if torch.is_grad_enabled() and self.graph != "sgangat" else None
        # both poolings in one launch (sgg_pool_fwd2): a's is held until b's carries it
        with K.pool_pair():
            with torch.no_grad():
                pool_a = self.pool_net(h_a, sse_a, obs_a[-1], scenes=sc_a, U=U_a)
            pool_b = self.pool_net(h_b, sse_b, obs_b[-1], scenes=sc_b, link=link, U=U_b)
        if self.graph == "sgangat":
            # both batches' batched-GAT layers, then both GCNModules, in
            # shared launches
            x_a, x_b = self.gatencoder.forward_pair((h_a.view(-1, H), pool_a), sc_a, (h_b.view(-1, H), pool_b), sc_b)
            comp = K.GcnModCompanion(x_a, g_a[-1], sc_a)
            y_b = self.gcn_module(x_b, sse_b, obs_b[-1], g_b[-1], scenes=sc_b, companion=comp)
            return comp.y, y_b
        if self.graph == "gat":
            comp = K.GatEncCompanion(h_a.view(-1, H), g_a[-1], sc_a, x2=pool_a)
            module = self.gatencoder
        else:
            comp = K.GcnModCompanion(h_a.view(-1, H), g_a[-1], sc_a, x2=pool_a)
            module = self.gcn_module
        y_b = module((h_b.view(-1, H), pool_b), sse_b, obs_b[-1], g_b[-1], scenes=sc_b, link=link, companion=comp)
        return comp.y, y_b

    def decode(self, noise_input, obs_traj, obs_traj_rel, seq_start_end, user_noise=None, *, scenes=None,
               copies=1, noise_index=None):
        """add_noise + decoder (models.py:909-925) for `copies` samples of the
        batch laid out sample-major (scene s of copy r is scene r*S + s, as
        SceneIndex.repeat builds it); user_noise then holds copies*S rows
        (global mix).  noise_index = (best, first_k): user_noise is the
        (K, S, nz) stack of K draws and copy r takes draw best[s] (r = 0, if
        best is given) or first_k + r (- 1 with best).
        -> pred_traj_fake_rel (pred_len, copies*B, 2)."""
        sc = _scenes(seq_start_end, obs_traj.device, scenes)
        if (not self.pool_every_timestep and self.noise_dim and self.noise_mix_type == "global"
                and user_noise is not None and self.num_layers == 1):
            # one launch builds h0 = [ctx | z_scene] and the first input for all copies
            nz = self.noise_first_dim
            if noise_index is None:
                z, best, first_k = user_noise.reshape(copies, sc.S, nz), None, 0
            else:
                (best, first_k), z = noise_index, user_noise
            z = z.to(noise_input.device, non_blocking=True)
            h0, rel0 = K.decoder_init(noise_input, z, best, first_k, copies, sc, obs_traj_rel[-1], lazy=True)
            with K.final_state_unused():   # (the decoder state is discarded, models.py:925)
                _h, rel = K.lstm_sequence(rel0, self.decoder.decoder, self.decoder.spatial_embedding, h0=h0, c0=None,
                                          proj=self.decoder.hidden2pos, decoder=True, T=self.pred_len)
            return rel
        if noise_index is not None and user_noise is not None:
            best, first_k = noise_index
            zk = user_noise.to(noise_input.device)
            ar = torch.arange(sc.S, device=zk.device)
            parts = [zk[best, ar]] if best is not None else []
            parts += [zk[first_k + r] for r in range(copies - len(parts))]
            user_noise = torch.cat(parts, 0)
        last_pos, last_rel = obs_traj[-1], obs_traj_rel[-1]
        if copies > 1:
            if self.pool_every_timestep:
                raise NotImplementedError("decode(copies>1) with per-step pooling: run forward() per sample")
            sc = sc.repeat(copies)
            noise_input = noise_input.repeat(copies, 1)
            last_pos, last_rel = last_pos.repeat(copies, 1), last_rel.repeat(copies, 1)
            seq_start_end = None
        decoder_h = self.add_noise(noise_input, seq_start_end, user_noise=user_noise, scenes=sc).unsqueeze(0)
        # c0 = 0 (models.py:912): the fused decoder takes a NULL initial cell
        # state as zeros; the per-step fallback needs the tensor
        decoder_c = (torch.zeros(self.num_layers, sc.B, self.decoder_h_dim, device=obs_traj.device)
                     if self.pool_every_timestep else None)
        out, _ = self.decoder(last_pos, last_rel, (decoder_h, decoder_c), seq_start_end, scenes=sc)
        return out


class TrajectoryDiscriminator(nn.Module):
    def __init__(self, obs_len, pred_len, embedding_dim=64, h_dim=64, mlp_dim=1024, num_layers=1,
                 activation="relu", batch_norm=True, dropout=0.0, d_type="local"):
        super().__init__()
        self.obs_len = obs_len
        self.pred_len = pred_len
        self.seq_len = obs_len + pred_len
        self.h_dim = h_dim
        self.d_type = d_type
        self.encoder = Encoder(embedding_dim=embedding_dim, h_dim=h_dim, mlp_dim=mlp_dim, num_layers=num_layers,
                               dropout=dropout)
        if d_type == "global":
            mlp_pool_dims = [h_dim + embedding_dim, mlp_dim, h_dim]
            self.pool_net = PoolHiddenNet(embedding_dim=embedding_dim, h_dim=h_dim, mlp_dim=mlp_pool_dims,
                                          bottleneck_dim=h_dim, activation=activation, batch_norm=batch_norm)
        self.real_classifier = make_mlp([h_dim, mlp_dim, 1], activation=activation, batch_norm=batch_norm,
                                        dropout=dropout)

    def fold_specs(self):
        """The discriminator's input-embedding folds (encoder, pooling)."""
        specs = [K.lstm_fold_spec(self.encoder.encoder, self.encoder.spatial_embedding)]
        if self.d_type != "local":
            specs.append(K.pool_fold_spec(self.pool_net))
        return specs

    def forward(self, traj, traj_rel, seq_start_end=None, *, scenes=None):
        if self.encoder.num_layers == 1:   # encoder + pooling folds in one launch (kernels.prefold)
            K.prefold(self.fold_specs())
        if self.d_type != "local" and self.encoder.num_layers == 1 and self.pool_net.fused_ok():
            # the pooling net's first layer (h half) in the encoder kernel's epilogue
            final_h, U = self.encoder(traj_rel, proj_u=K.pool_u_spec(self.pool_net))
        else:
            final_h, U = self.encoder(traj_rel), None
        if self.d_type == "local":
            x = final_h.squeeze()
        else:
            x = self.pool_net(final_h.squeeze(), seq_start_end, traj[0], scenes=scenes, U=U)
        # Linear -> ReLU -> Linear(., 1) -> ReLU in one launch each way
        spec = K.head_ok(self.real_classifier)
        if spec is not None and x.dim() == 2:
            return K.head(x, spec)
        return run_mlp(self.real_classifier, x)
