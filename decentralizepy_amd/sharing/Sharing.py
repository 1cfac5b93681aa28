"""Sharing plugin (full-model gossip) over the MI355X codec.

Drop-in for the reference ``decentralizepy.sharing.Sharing.Sharing``
(``src/decentralizepy/sharing/Sharing.py``): same constructor keyword arguments, same methods and
attributes used by the Node code (``get_data_to_send``, ``_averaging``, ``_averaging_server``,
``_pre_step``, ``_post_step``, ``serialized_model``, ``deserialized_model``, ``compress_data``,
``decompress_data``, ``communication_round``).  Payload dicts on the wire keep the reference
format (numpy arrays + scalars), so ``communication.TCP`` and the Node code run unchanged.

What runs on the GPU: the Metro-Hastings fold of the received models (``_averaging``) is one
``dpz_decode_average`` launch over all payloads (HIP kernel ``fold_kernel``), bit-exact with the
reference's per-key fp32 fold (``Sharing.py:156-190``).
"""
import importlib
import logging

import numpy as np
import torch

from .. import codec
from .._device import (PayloadNames, Staging, flatten_state, h2d_array, load_flat,
                       pick_device, state_to_device, to_host)


class Sharing:
    """API defining who to share with and what, and what to do on receiving."""

    def __init__(self, rank, machine_id, communication, mapping, graph, model, dataset, log_dir,
                 compress=False, compression_package=None, compression_class=None,
                 float_precision=None):
        # reference Sharing.py:13-78
        self.rank = rank
        self.machine_id = machine_id
        self.uid = mapping.get_uid(rank, machine_id)
        self.communication = communication
        self.mapping = mapping
        self.graph = graph
        self.model = model
        self.dataset = dataset
        self.communication_round = 0
        self.log_dir = log_dir

        self.shapes = []
        self.lens = []
        with torch.no_grad():
            for _, v in self.model.state_dict().items():
                self.shapes.append(v.shape)
                self.lens.append(v.numel())
        self.number_of_params = int(sum(self.lens))

        self.compress = compress
        if compression_package and compression_class:
            compressor_module = importlib.import_module(compression_package)
            compressor_class = getattr(compressor_module, compression_class)
            self.compressor = compressor_class(float_precision=float_precision)
            logging.debug(f"Using the {compressor_class} to compress the data")
        else:
            assert not self.compress

        self.device = pick_device(rank)
        self.staging = Staging()
        self._pay_names = PayloadNames()
        self.workspace = codec.Workspace(self.device)
        self._recv_status = None  # the round's asynchronous-decode status word
        self._recv_status_used = False
        if hasattr(getattr(self, "compressor", None), "_dev"):
            self.compressor.device = self.device  # device compressors run on this node's GPU

    # ---- wire format -----------------------------------------------------------------------
    def compress_data(self, data):
        result = dict(data)
        if self.compress:
            if "params" in result:
                result["params"] = self.compressor.compress_float(result["params"])
        return result

    def decompress_data(self, data, device=False):
        if self.compress:
            if "params" in data:
                if device and hasattr(self.compressor, "decompress_float_device"):
                    data["params"] = self.compressor.decompress_float_device(data["params"])
                else:
                    data["params"] = self.compressor.decompress_float(data["params"])
        return data

    def serialized_model(self):
        """Full flat model as numpy (reference Sharing.py:93-112)."""
        with torch.no_grad():
            flat = flatten_state(self.model.state_dict())
        data = {"params": flat.numpy()}
        return self.compress_data(data)

    def deserialized_model(self, m):
        """Received dict -> state_dict of CPU tensors (reference Sharing.py:114-140)."""
        m = self.decompress_data(m)
        return self._unflatten(np.asarray(m["params"]))

    def _unflatten(self, flat):
        state_dict = dict()
        start = 0
        for i, key in enumerate(self.model.state_dict()):
            end = start + self.lens[i]
            state_dict[key] = torch.from_numpy(np.asarray(flat[start:end]).reshape(self.shapes[i]))
            start = end
        return state_dict

    # ---- round hooks ------------------------------------------------------------------------
    def _pre_step(self):
        pass

    def _post_step(self):
        pass

    def get_data_to_send(self, degree=None):
        """reference Sharing.py:192-198"""
        self._pre_step()
        data = self.serialized_model()
        my_uid = self.mapping.get_uid(self.rank, self.machine_id)
        data["degree"] = degree if degree != None else len(self.graph.neighbors(my_uid))  # noqa: E711
        data["iteration"] = self.communication_round
        return data

    # ---- receive side -------------------------------------------------------------------------
    def _local_flat_device(self):
        """Current local model as a flat fp32 device vector (the fold's local term)."""
        with torch.no_grad():
            return state_to_device(self.model.state_dict(), self.device, self.staging, "local")

    def _h2d(self, arr, dtype, leg):
        """A host payload leg to the device through a pinned buffer (async DMA, overlapping the
        host work on the next payload); device tensors (decoded by a device compressor) stay."""
        if isinstance(arr, torch.Tensor):
            return arr.to(self.device, torch.from_numpy(np.zeros(0, dtype)).dtype).reshape(-1)
        return h2d_array(arr, dtype, self.device, self.staging, self._pay_names(leg))

    def _device_payload(self, data):
        """Received (decompressed) payload dict -> (idx int32 device or None, vals fp32 device)."""
        return None, self._h2d(data["params"], np.float32, "params")

    def _recv_status_word(self):
        """The round's device status word for asynchronous payload decodes (zeroed on first use
        in a round; ``_check_received`` reads it once)."""
        if getattr(self, "_recv_status", None) is None:
            self._recv_status = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._recv_status_used = False
        if not self._recv_status_used:
            self._recv_status.zero_()
            self._recv_status_used = True
        return self._recv_status

    def _check_received(self):
        """Raise if an asynchronous payload decode of this round saw a malformed stream (one
        synchronisation: the fold output is read back right after anyway)."""
        if getattr(self, "_recv_status_used", False):
            self._recv_status_used = False
            if int(self._recv_status.item()) != 0:
                raise ValueError("malformed payload stream (Elias or float leg)")

    def _pop_payloads(self, peer_deques):
        payloads, degrees = [], []
        for n in peer_deques:
            data = peer_deques[n].popleft()
            degree, iteration = data["degree"], data["iteration"]
            del data["degree"]
            del data["iteration"]
            del data["CHANNEL"]
            logging.debug("Averaging model from neighbor {} of iteration {}".format(n, iteration))
            data = self.decompress_data(data, device=True)
            payloads.append(self._device_payload(data))
            degrees.append(degree)
        return payloads, degrees

    def _fold(self, local, payloads, weights, w_self):
        out = torch.empty_like(local)
        return codec.decode_average(local, payloads, weights, w_self, out=out,
                                    workspace=self.workspace)

    def _load_flat(self, out_dev):
        self._check_received()
        # load_state_dict of the averaged model with its D2H pipelined against the host copy
        load_flat(self.model, out_dev, self.staging, "result")

    def _averaging(self, peer_deques):
        """Metro-Hastings average of the received models with the local one
        (reference Sharing.py:156-190; one batched fold kernel over all payloads)."""
        with torch.no_grad():
            payloads, degrees = self._pop_payloads(peer_deques)
            weights = [1 / (max(len(peer_deques), d) + 1) for d in degrees]
            weight_total = 0
            for w in weights:
                weight_total += w
            local = self._local_flat_device()
            out = self._fold_on_base(local, payloads, weights, 1 - weight_total)
            if out is None:
                out = self._fold(local, payloads, weights, 1 - weight_total)
            self._load_flat(out)
        self._post_step()
        self.communication_round += 1

    def _fold_on_base(self, local, payloads, weights, w_self):
        """The fold over a no-hit base the encode already wrote (PartialModel), or None."""
        return None

    def _averaging_server(self, peer_deques):
        """Plain average of the working nodes' models (reference Sharing.py:200-229)."""
        with torch.no_grad():
            payloads, _ = self._pop_payloads(peer_deques)
            weights = [1 / len(peer_deques)] * len(payloads)
            local = self._local_flat_device()
            out = self._fold(local, payloads, weights, None)
            self._check_received()
            flat = to_host(out, self.staging, "result")
            total = self._unflatten(flat)
        self.model.load_state_dict(total)
        self._post_step()
        self.communication_round += 1
        return total
