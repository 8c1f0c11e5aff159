"""Helpers shared by the multi-process tests (gloo on the CPU, or ranks sharing one GPU)."""
import socket


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
