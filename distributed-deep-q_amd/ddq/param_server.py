"""Parameter server with the semantics of param-server/server.py (reference),
its model and optimizer state resident on the GPU.

Endpoints (server.py:181-215) as methods -- ``get_model_params`` (GET
/api/v1/latest_model), ``update_params`` (POST /api/v1/update_model),
``clear_params`` (GET /api/v1/clear_model) -- plus ``serve(port)``, a stdlib
HTTP front end with the same routes and ``application/deepQ`` bodies, so an
unmodified reference worker can talk to it.

Semantics kept:
* the central model holds the ``Q*`` parameters; a pull at
  ``iteration % special_update_period == 0`` first copies Q -> P
  (server.py:127-137, :188-189), after which P* blobs are part of every
  model message (dict order: Q* then P*);
* a push increments ``iteration`` then applies the gradient with the selected
  rule -- sgd (:81-83), rmsprop with the one-step-lagged cache (:86-105,
  default), adagrad (:108-124) -- each on arrival, i.e. with the reference's
  unbounded staleness;
* ``snapshot_frequency`` (:74-77): every that many iterations the model is
  handed to ``on_snapshot(name, params)`` (Celery's ``saveSnapshot`` in the
  reference; a callback here).
The apply runs in ``apply_kernel`` on the device (``ddq_set_grads`` +
``ddq_apply``), not in numpy.
"""
from __future__ import annotations

import pickle
import struct
import threading

import numpy as np

from . import params as P
from .barista import messaging
from .net import DeepQNet

MODEL_NAME = "centralModel"     # server.py:13


def get_snapshot_name(iteration):
    return MODEL_NAME + "-%06d" % iteration     # server.py:41-42


class ParamServer:
    def __init__(self, frame=16, batch=32, update="rmsprop", lr=1e-4, rmsprop_decay=0.9,
                 special_update=10, snapshot_freq=500, stats_freq=500, device=0,
                 on_snapshot=None, mode="gpu"):
        if update not in ("sgd", "rmsprop", "adagrad"):
            raise ValueError("update must be one of adagrad, rmsprop, sgd")
        self.net = DeepQNet(batch=batch, frame=frame, device=device, mode=mode)
        self.update = update
        self.learning_rate = float(lr)
        self.rmsprop_decay = float(rmsprop_decay)
        self.special_update_period = int(special_update)
        self.snapshot_frequency = int(snapshot_freq)
        self.stats_frequency = int(stats_freq)
        self.on_snapshot = on_snapshot
        self.iteration = 0
        self.has_model = False
        self.has_target = False
        self.model_lock = threading.Lock()

    # server.py:218-257 initParams(reset=True)
    def init_params(self, params=None, seed=42):
        """Model from ``params`` ({Q*: [W, b]}) or the prototxt fillers."""
        with self.model_lock:
            if params is None:
                params = P.init_params(self.net.frame, seed=seed)
            self.net.set_flat(0, self.net.join(params, "Q"))
            self.net.reset_optimizer()
            self.iteration = 0
            self.has_model = True
            self.has_target = False

    def clear_params(self):
        """GET /api/v1/clear_model (server.py:212-215)."""
        with self.model_lock:
            self.has_model = False
            self.has_target = False
        return b"Cleared"

    def model_params(self):
        out = self.net.split(self.net.get_flat(0), "Q")
        if self.has_target:
            out.update(self.net.split(self.net.get_flat(1), "P"))
        return out

    def get_model_params(self):
        """GET /api/v1/latest_model (server.py:181-193) -> model message bytes."""
        with self.model_lock:
            if not self.has_model:
                return messaging.create_message({}, self.iteration)
            if self.iteration % self.special_update_period == 0:
                self.net.sync_target()
                self.has_target = True
            return messaging.create_message(self.model_params(), self.iteration)

    def update_params(self, message):
        """POST /api/v1/update_model (server.py:196-209) -> b"Updated"."""
        grads = messaging.load_gradient_message(message)
        missing = [k for k in self.net.q_names if k not in grads]
        if missing:
            # server.py:86-124 would touch only the received keys; workers
            # always send every Q blob (messaging.py:43-79), and the device
            # apply updates the whole tower -- a partial message is refused
            # rather than zero-filled (which would still decay the rmsprop
            # cache / consume adagrad's first call of the missing blobs)
            raise ValueError("gradient message lacks %s" % ", ".join(missing))
        with self.model_lock:
            self.iteration += 1
            flat = self.net.join({k: v for k, v in grads.items()}, "Q")
            self.net.set_grads_flat(flat)
            self.net.apply(self.update, lr=self.learning_rate, decay=self.rmsprop_decay)
            if self.snapshot_frequency and self.iteration % self.snapshot_frequency == 0 \
                    and self.on_snapshot is not None:
                self.on_snapshot(get_snapshot_name(self.iteration), self.model_params())
        return b"Updated"

    # ---------------------------------------------------------------- HTTP
    def serve(self, port=5500, host="127.0.0.1"):
        """Blocking HTTP server with the reference's routes (server.py:165-215)."""
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        ps = self

        class Handler(BaseHTTPRequestHandler):
            def _reply(self, body, status=200):
                self.send_response(status)
                self.send_header("Content-Type", "application/deepQ")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path == "/api/v1/latest_model":
                    self._reply(ps.get_model_params())
                elif self.path == "/api/v1/clear_model":
                    self._reply(ps.clear_params())
                elif self.path == "/":
                    self._reply(b"Param Server")
                else:
                    self._reply(b"not found", 404)

            def do_POST(self):
                if self.path != "/api/v1/update_model":
                    return self._reply(b"not found", 404)
                n = int(self.headers.get("Content-Length", "0"))
                try:
                    body = ps.update_params(self.rfile.read(n))
                except (ValueError, KeyError, struct.error, pickle.UnpicklingError) as e:
                    return self._reply(("bad gradient message: %s" % e).encode(), 400)
                self._reply(body)

            def log_message(self, *args):
                pass

        httpd = ThreadingHTTPServer((host, port), Handler)
        self._httpd = httpd
        try:
            httpd.serve_forever()
        finally:
            httpd.server_close()

    def shutdown(self):
        if getattr(self, "_httpd", None) is not None:
            self._httpd.shutdown()
