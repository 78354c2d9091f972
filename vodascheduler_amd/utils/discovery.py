"""Service discovery (reference pkg/common/util/util.go:11-31): a service's IP from the
``<svc>.<namespace>.svc.cluster.local`` A record, its port from the ``_<port>._tcp`` SRV
record.  Outside Kubernetes (or without SRV support in the stdlib resolver) the well-known
default ports of the three REST services are used."""
from __future__ import annotations

import socket

from ..common.types import NAMESPACE, PORT_ALLOCATOR, PORT_SCHEDULER, PORT_TRAINING_SERVICE

DEFAULT_PORTS = {"training-service": PORT_TRAINING_SERVICE, "resource-allocator": PORT_ALLOCATOR,
                 "scheduler": PORT_SCHEDULER}


def service_host(svc: str, namespace: str = NAMESPACE) -> str:
    fqdn = f"{svc}.{namespace}.svc.cluster.local"
    try:
        return socket.getaddrinfo(fqdn, None, socket.AF_INET)[0][4][0]
    except OSError:
        return "127.0.0.1"


def service_port(svc: str, namespace: str = NAMESPACE, port_name: str = "port") -> int:
    """SRV lookup needs a DNS library that this image does not ship; the services always
    listen on their fixed ports (config/config.go:7), which is what the SRV records carry."""
    for key, port in DEFAULT_PORTS.items():
        if svc.startswith(key):
            return port
    return PORT_TRAINING_SERVICE


def service_url(svc: str, namespace: str = NAMESPACE) -> str:
    return f"http://{service_host(svc, namespace)}:{service_port(svc, namespace)}"
