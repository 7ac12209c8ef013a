"""DCN-v2 cross network of ``DLRMTrainer`` (mixin): x_{l+1} = x0 * (U (V^T
x_l) + b) + x_l, the explicit forward / backward of the cross layers on the
fused HIP GEMM epilogues (the role of the reference's ``torchrec`` DCN model,
SURVEY.md NS3)."""
from __future__ import annotations

from .. import ops


class DCNMixin:
    """Cross-layer forward / backward; the buffers and layers (``dcn_x``,
    ``dcn_h``, ``dcn_y``, ``dcn_u``, ...) are set up by ``DLRMTrainer``."""

    # DCN-v2 cross network: x_{l+1} = x0 * (U (V^T x_l) + b) + x_l. The
    # Hadamard product and the residual are fused into the U-GEMM epilogue
    # (out2 = x0 * (acc + b) + x_l), the residual of the backward into the
    # V-dgrad epilogue.
    def _dcn_forward(self, h):
        cfg, fp, D, F = self.cfg, self.fp, self.cfg.embedding_dim, self.F
        Wd = self.top_real
        x0 = self.dcn_x[0]
        if not self._x0_alias:
            ops.concat_features(h, self.emb.recv, self.slot_off, self.slot_stride, F, D, x0)
        for i in range(cfg.dcn_layers):
            u = self.dcn_u[i]
            ops.linear_fwd(self.dcn_x[i][:, :Wd], fp.bf16(f"dcn{i}.v"), None, relu=False,
                           out=self.dcn_h[i][:, :u.in_real])
            Uw = fp.bf16(u.name + ".w")
            ops.gemm(self.dcn_h[i][:, :u.in_k], False, Uw[:, :u.in_k], False,
                     None if u.bias_in_k else fp.param(u.name + ".w")[:, u.bcol], False, None,
                     self.dcn_y[i], None, 1, mul=x0, add=self.dcn_x[i][:, :Wd],
                     out2=self.dcn_x[i + 1][:, :Wd])

    def _dcn_backward(self, h):
        cfg, fp, D, F = self.cfg, self.fp, self.cfg.embedding_dim, self.F
        Lc = cfg.dcn_layers
        x0 = self.dcn_x[0]
        acc = self.dcn_dx0acc
        for i in reversed(range(Lc)):
            u = self.dcn_u[i]
            dxo = self.dcn_dx[i + 1]
            dy, dh = self._dcn_bufs(i)
            # dy = dxo * x0 ; acc (+)= dxo * y (+ dxo at i == 0: x_0's residual)
            ops.cross_bwd(dxo, x0, self.dcn_y[i], dy, acc, i != Lc - 1, i == 0)
            Uw = fp.bf16(u.name + ".w")
            # U's weight grad and dgrad (both read dy): one paired launch
            with ops.gemm_batch(self._pair_bwd and not self._defer_top_wgrad):
                if not self._defer_top_wgrad:
                    self._wgrad_gemm(u, self.dcn_h[i], dy)
                ops.gemm(dy, False, Uw[:, :u.in_k], True, None, False, None, dh, None, 1)
            # V's weight grad and dgrad (both read dh): one paired launch
            with ops.gemm_batch(self._pair_bwd and not self._defer_top_wgrad
                                and f"dcn{i}.v" in self.wslab):
                if not self._defer_top_wgrad:
                    self._dcn_wgrad_v(i)
                # dx_i = dh V + (i > 0 ? dxo : acc)
                ops.gemm(dh, False, fp.bf16(f"dcn{i}.v"), True, None, False, None, None, None,
                         1, add=dxo if i > 0 else acc, out2=self.dcn_dx[i])
        if self._x0_alias:      # only the dense slot's ReLU-masked gradient
            ops.split_features(self.dcn_dx[0], 1, D, h, self.bot_grad[-1], self.emb.d_recv,
                               self.slot_off, self.slot_stride, True)
        else:
            ops.split_features(self.dcn_dx[0], F, D, h, self.bot_grad[-1], self.emb.d_recv,
                               self.slot_off, self.slot_stride, True)

    def _dcn_bufs(self, i: int):
        j = i if len(self.dcn_dyl) > 1 else 0
        return self.dcn_dyl[j], self.dcn_dhl[j]

    def _dcn_wgrad_v(self, i: int):
        """dV_i = dh_i^T x_i (split-K partials summed by the optimizer on one
        GPU, with their all-reduce bucket otherwise: DLRMTrainer._reduce_slabs)."""
        _, dh = self._dcn_bufs(i)
        Wd = self.top_real
        if f"dcn{i}.v" in self.wslab:
            sl, S = self.wslab[f"dcn{i}.v"]
            ops.gemm(dh, True, self.dcn_x[i][:, :Wd], True, None, False, None, None, sl, S)
        else:
            ops.linear_wgrad(dh, self.dcn_x[i][:, :Wd], self.fp.grad(f"dcn{i}.v").view(-1),
                             splits=self._wg_splits(self.cfg.dcn_rank, Wd), slab=self.slab)
