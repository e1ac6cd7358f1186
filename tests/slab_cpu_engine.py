"""CPU pass engine for hipgp_amd.slab (TEST INFRASTRUCTURE): the reference's own operator
definition (`toeplitz_tensor.py:70-125`: pad -> FFT_n -> x spectrum -> IFFT_n -> crop on the
circulant n-grid, spectrum D / 1/D / sqrt(D) of the oracle) split into the same three slab
stages as libhipgp's hgp_slab_pass, over the same exchange-layout contract E[g][q][i][c]
(here: d = 2 g = rfft column of axis 1, inner 1; d = 3 g = axis-1 frequency, c = rfft column
of axis 2).  Lets the gloo tests check the partition / all-to-all / all-reduce logic of
SlabToeplitz on the CPU against the oracle."""
import numpy as np
import torch

from hipgp_amd import _lib


class CpuSlabEngine:
    def __init__(self, T):
        """T: oracle.ziggy_oracle.ToeplitzOracle of the whole grid."""
        self.T = T
        self.dims = T.dims
        self.n = tuple(T.ndims)
        self.d = len(self.dims)
        self.dtype = torch.float64 if T.dtype == np.float64 else torch.float32
        self.cdtype = torch.complex128 if self.dtype == torch.float64 else torch.complex64
        self.spec = {_lib.OP_K: T.D, _lib.OP_CINV: T.Di, _lib.OP_RT: T.D_sqrt, _lib.OP_R: T.D_sqrt}

    def geometry(self, op):
        if self.d == 2:
            return self.n[1] // 2 + 1, 1
        return self.n[1], self.n[2] // 2 + 1

    def _io(self, op):
        ins = self.n if op == _lib.OP_R else self.dims
        outs = self.n if op == _lib.OP_RT else self.dims
        return ins, outs

    @staticmethod
    def _masked(done):
        return done is not None and int(done.reshape(-1)[0]) != 0

    def fwd(self, op, x, nrows, E, done=None):
        if self._masked(done):
            return
        ins, _ = self._io(op)
        xv = x.detach().cpu().numpy().reshape((x.shape[0], nrows) + tuple(ins[1:]))
        if self.d == 2:
            F = np.fft.rfft(xv, n=self.n[1], axis=2)                    # (q, i, g)
            E.copy_(torch.from_numpy(np.ascontiguousarray(F.transpose(2, 0, 1)[..., None])))
        else:
            F = np.fft.rfft(xv, n=self.n[2], axis=3)
            F = np.fft.fft(F, n=self.n[1], axis=2)                      # (q, i, k1, c2)
            E.copy_(torch.from_numpy(np.ascontiguousarray(F.transpose(2, 0, 1, 3))))

    def conv(self, op, lines, g0, ng, nrhs):
        ins, outs = self._io(op)
        L = lines.cpu().numpy()[:, :, :ins[0], :]                        # (g, q, in0, c)
        F = np.fft.fft(L, n=self.n[0], axis=2)
        S = self.spec[op]
        if self.d == 2:
            s = S[:, g0:g0 + ng].T[:, None, :, None]                     # (g, 1, k0, 1)
        else:
            s = S[:, g0:g0 + ng, :self.n[2] // 2 + 1].transpose(1, 0, 2)[:, None]   # (g, 1, k0, c2)
        Y = np.fft.ifft(F * s, axis=2)[:, :, :outs[0], :]
        lines[:, :, :outs[0], :] = torch.from_numpy(np.ascontiguousarray(Y))

    @staticmethod
    def _blocks(total, ws):
        """The balanced row split of hipgp_amd.slab.split, as (start, count) per rank."""
        base, rem = divmod(total, ws)
        out, a = [], 0
        for r in range(ws):
            c = base + (1 if r < rem else 0)
            out.append((a, c))
            a += c
        return out

    def conv_a2a(self, op, recv, send, g0, ng, nrhs, ws, done=None):
        """HGP_SLAB_CONV_A2A: lines read from the receive buffer's rank blocks
        [r][g][q][i - a_r][c], results written to the send buffer's [r][g][q][o - b_r][c]."""
        if self._masked(done):
            return
        ins, outs = self._io(op)
        _, inner = self.geometry(op)
        lines = torch.zeros((ng, nrhs, max(ins[0], outs[0]), inner), dtype=self.cdtype)
        R = recv.cpu()
        off = 0
        for a, c in self._blocks(ins[0], ws):
            n = ng * nrhs * c * inner
            lines[:, :, a:a + c, :] = R[off:off + n].view(ng, nrhs, c, inner)
            off += n
        self.conv(op, lines, g0, ng, nrhs)
        off = 0
        for b, c in self._blocks(outs[0], ws):
            n = ng * nrhs * c * inner
            send[off:off + n] = lines[:, :, b:b + c, :].reshape(-1).to(send.device)
            off += n

    def inv(self, op, E, nrows, y, dotv=None, dot_out=None, done=None):
        if self._masked(done):
            return
        _, outs = self._io(op)
        A = E.cpu().numpy()
        if self.d == 2:
            Y = np.fft.irfft(A[..., 0].transpose(1, 2, 0), n=self.n[1], axis=2)[..., :outs[1]]
        else:
            B = np.fft.ifft(A.transpose(1, 2, 0, 3), n=self.n[1], axis=2)
            Y = np.fft.irfft(B, n=self.n[2], axis=3)[:, :, :outs[1], :outs[2]]
        y.copy_(torch.from_numpy(np.ascontiguousarray(Y.reshape(y.shape))))
        if dotv is not None:
            dot_out.copy_((y * dotv).sum(dim=1))

    # -- the slab PCG's updates (the contract of hgp_slab_cg_*: dots already all-reduced) ----
    def dot(self, a, c, out):
        out.copy_((a * c).sum(dim=1))

    def cg_xr(self, x, r, p, Ap, rs, pAp, rr, done):
        if self._masked(done):
            return
        al = (rs / pAp).unsqueeze(-1)
        x += al * p
        r -= al * Ap
        rr.copy_((r * r).sum(dim=1))

    def cg_check(self, rr, tol, done, iters):
        if self._masked(done):
            return
        iters += 1
        if bool(torch.all(torch.sqrt(rr) < tol)):
            done.copy_(iters)

    def cg_p(self, p, z, rs, zr, done):
        if self._masked(done):
            return
        beta = (zr / rs).unsqueeze(-1)
        rs.copy_(zr)
        p.mul_(beta).add_(z)
