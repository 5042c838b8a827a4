"""Fake Spark executor (barista/dummy_client.py, reference): connect to a
Barista worker, send one request byte, read the reply until EOF.

    python -m ddq.barista.dummy_client [N] [--port 50001]
"""
import socket
import sys

from . import GRAD_UPDATE


class DummyClient:
    def __init__(self, address, port):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.connect((address, port))

    def send(self, msg):
        total = 0
        while total < len(msg):
            sent = self.sock.send(msg[total:])
            if sent == 0:
                raise RuntimeError("socket connection broken")
            total += sent

    def recv(self, bufsize=1024):
        response = b""
        while True:
            chunk = self.sock.recv(bufsize)
            if not chunk:
                break
            response += chunk
        return response

    def close(self):
        self.sock.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    port = 50001
    if "--port" in argv:
        i = argv.index("--port")
        port = int(argv[i + 1])
        del argv[i:i + 2]
    n = int(argv[0]) if argv else 1
    for i in range(n):
        c = DummyClient("127.0.0.1", port)
        c.send(GRAD_UPDATE)
        print("Response[%d]:" % i, c.recv().decode(errors="replace"))
        c.close()


if __name__ == "__main__":
    main()
