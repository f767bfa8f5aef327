"""JSON-lines TCP server with the reference's socket protocol, backed by the GPU batch.

SURVEY §8(f) row 4: a drop-in for ``delivery_drone/socket_server.py`` +
``game/socket_server.py:126-263`` (protocol: ``SOCKET_API.md:65-196``) for
remote or legacy clients.  The reference's own ``DroneGameClient``
(``game/socket_client.py``) connects to it unchanged:

* on connect the server sends ``{"type": "HANDSHAKE", "num_games": N}``;
* requests are one JSON object per line: ``RESET`` / ``STEP`` (with
  ``action``) / ``GET_STATE`` with ``game_id`` (default 0), and ``CLOSE``;
* answers are ``{"type": "STATE", "game_id", "state", "reward", "done",
  "info"}`` or ``{"type": "ERROR", "message"}``, with the reference's messages
  for a bad ``game_id``, an unknown type and invalid JSON.

Every game is one lane of a :class:`VecDroneEnv` with ``auto_reset=False``
(the reference's sticky done: a STEP after the end returns reward 0, done
True and ``info["needs_reset"]``).  The reference serves one client and runs
its command loop at a fixed frame rate (``--fps``, default 60); this server
answers each request as soon as its kernel has run, and serves any number of
clients (commands are serialised on the batch).

    python -m delivery_drone_amd.server --num-games 16 --port 5555 [--randomize-drone] [--fixed-spawn]
"""
from __future__ import annotations

import argparse
import json
import socket
import threading
from typing import Optional

from .compat import _Lanes
from .vec_env import VecDroneEnv

__all__ = ["BatchSocketServer", "main"]


class BatchSocketServer:
    """Serve the lanes of ``env`` over the reference's socket protocol.

    ``port=0`` binds an ephemeral port (see :attr:`port` after :meth:`start`).
    """

    def __init__(self, env: VecDroneEnv, host: str = "127.0.0.1", port: int = 5555):
        if env.config.auto_reset:
            raise ValueError("the socket protocol needs auto_reset=False (clients send RESET)")
        self.env = env
        self.num_games = env.num_envs
        self.host, self.port = host, port
        self._lanes = _Lanes(env)
        self._lock = threading.Lock()
        self._sock: Optional[socket.socket] = None
        self._threads = []
        self.running = False
        self.requests = 0

    # -- lifecycle ---------------------------------------------------------
    def start(self) -> "BatchSocketServer":
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((self.host, self.port))
        s.listen(16)
        s.settimeout(0.2)
        self.port = s.getsockname()[1]
        self._sock = s
        self.running = True
        t = threading.Thread(target=self._accept_loop, name="dd-accept", daemon=True)
        t.start()
        self._threads.append(t)
        return self

    def stop(self):
        self.running = False
        for t in self._threads:
            t.join(timeout=2.0)
        if self._sock is not None:
            self._sock.close()
            self._sock = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _accept_loop(self):
        while self.running:
            try:
                conn, _ = self._sock.accept()
            except socket.timeout:
                continue
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            t = threading.Thread(target=self._serve, args=(conn,), name="dd-client", daemon=True)
            t.start()
            self._threads.append(t)

    # -- one client --------------------------------------------------------
    def _serve(self, conn: socket.socket):
        conn.settimeout(0.2)
        buf = b""
        try:
            self._send(conn, {"type": "HANDSHAKE", "num_games": self.num_games})
            while self.running:
                try:
                    data = conn.recv(65536)
                except socket.timeout:
                    continue
                if not data:
                    break
                buf += data
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    line = line.strip()
                    if line and not self._handle(conn, line.decode("utf-8")):
                        return
        except OSError:
            pass
        finally:
            conn.close()

    @staticmethod
    def _send(conn, message: dict):
        conn.sendall((json.dumps(message) + "\n").encode("utf-8"))

    def _error(self, conn, text: str):
        self._send(conn, {"type": "ERROR", "message": text})

    def _handle(self, conn, line: str) -> bool:
        """One request (game/socket_server.py:126-188, 190-223); False = CLOSE."""
        try:
            msg = json.loads(line)
        except json.JSONDecodeError as e:
            self._error(conn, f"Invalid JSON: {e}")
            return True
        try:
            kind = msg.get("type")
            g = msg.get("game_id", 0)
            if g < 0 or g >= self.num_games:
                self._error(conn, f"Invalid game_id: {g}. Must be in range [0, {self.num_games})")
                return True
            if kind == "CLOSE":
                return False
            with self._lock:
                self.requests += 1
                if kind == "RESET":
                    state, reward, done, info = self._lanes.reset(g), 0.0, False, {}
                elif kind == "STEP":
                    state, reward, done, info = self._lanes.step(g, msg.get("action", {}))
                elif kind == "GET_STATE":
                    state, done, info = self._lanes.get_state_info(g)
                    reward = 0.0
                else:
                    self._error(conn, f"Unknown message type: {kind}")
                    return True
            self._send(conn, {"type": "STATE", "game_id": g, "state": state, "reward": float(reward),
                              "done": bool(done), "info": info})
        except Exception as e:  # the reference answers every failure with an ERROR line
            self._error(conn, f"Error handling message: {e}")
        return True


def main(argv=None):
    """Command line of the reference's ``delivery_drone/socket_server.py`` (headless)."""
    p = argparse.ArgumentParser(description="Delivery Drone socket server on the GPU batch")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=5555)
    p.add_argument("--render", choices=("none",), default="none", help="rendering is out of scope")
    p.add_argument("--num-games", type=int, default=1)
    p.add_argument("--randomize-drone", action="store_true")
    p.add_argument("--randomize-platform", action="store_true", default=True)
    p.add_argument("--fixed-spawn", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--precision", choices=("f32", "f64"), default="f64")
    args = p.parse_args(argv)
    rd, rp = (False, False) if args.fixed_spawn else (args.randomize_drone, args.randomize_platform)
    env = VecDroneEnv(args.num_games, randomize_drone=rd, randomize_platform=rp, auto_reset=False,
                      seed=args.seed, precision=args.precision)
    env.reset()  # the reference resets every game before serving (socket_server.py:147-148)
    server = BatchSocketServer(env, args.host, args.port).start()
    print(f"serving {args.num_games} game(s) on {args.host}:{server.port}", flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass
    finally:
        server.stop()


if __name__ == "__main__":
    main()
