"""The Kano paper's five-container cluster (kano_py/sample/example.py:4-60):
Nginx -> DB, User -> Tomcat, Tomcat -> Nginx, all as ingress policies.
Known answers: SURVEY.md §A.5 (checked against kano_py in tests/golden)."""
from kano.model import (Container, Policy, PolicyAllow, PolicyIngress, PolicyProtocol,
                        PolicySelect)

_CONTAINERS = [  # name, app, role
    ("A", "Alice", "Nginx"),
    ("B", "Alice", "DB"),
    ("C", "Alice", "Tomcat"),
    ("D", "Bob", "Nginx"),
    ("E", "User", "User"),
]

_POLICIES = [  # name, podSelector, ingress peer, port
    ("A", {"role": "DB"}, {"role": "Nginx"}, "3306"),
    ("B", {"role": "Tomcat"}, {"role": "User"}, "8080"),
    ("C", {"role": "Nginx"}, {"role": "Tomcat"}, "3306"),
    ("D", {"role": "Nginx"}, {"app": "Alice"}, "3306"),
]


def paper_example():
    containers = [Container(name, {"app": app, "role": role}) for name, app, role in _CONTAINERS]
    policies = [Policy(name, PolicySelect(dict(sel)), PolicyAllow(dict(peer)), PolicyIngress,
                       PolicyProtocol(["TCP", port]))
                for name, sel, peer, port in _POLICIES]
    return containers, policies
