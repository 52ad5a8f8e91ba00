"""Random REST rule sets that exercise every compiler quirk of SURVEY.md §8a
(non-octet prefixes Q6, colliding trie keys Q7, port-0 wildcard Q8, interface
wildcard Q9, negated-only tcpflags Q10, protocol fallback Q11, ...)."""
import random

FLAGS = ["FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"]
PORTS = {"veth1": 1, "veth2": 2, "eth0": 3, "lo": 0xFFFF}


def _ip(rnd, pool):
    return rnd.choice(pool)


def quirky_rules(n, seed, *, p_field=0.5, ct=True, ifaces=True, ip_pool=None):
    rnd = random.Random(seed)
    if ip_pool is None:
        ip_pool = []
        for _ in range(max(4, n // 3)):
            ln = rnd.choice([0, 1, 7, 8, 9, 12, 16, 19, 20, 23, 24, 25, 31, 32, 32])
            octs = [rnd.choice([10, 10, 192, 172, rnd.randrange(256)]), rnd.randrange(4),
                    rnd.choice([0, 16, 32, 48, rnd.randrange(256)]), rnd.randrange(256)]
            ip_pool.append(".".join(map(str, octs)) + ("" if ln == 32 and rnd.random() < 0.3 else f"/{ln}"))
    port_pool = [0, 0, 22, 53, 80, 443, 8080, 65535, rnd.randrange(65536)]
    rules = []
    for _ in range(n):
        r = {}
        if rnd.random() < p_field:
            r["src"] = _ip(rnd, ip_pool)
        if rnd.random() < p_field:
            r["dst"] = _ip(rnd, ip_pool)
        if rnd.random() < p_field:
            r["l4proto"] = rnd.choice(["TCP", "UDP", "ICMP", "GRE", "tcp", "udp"])
        if rnd.random() < p_field * 0.6:
            r["sport"] = rnd.choice(port_pool)
        if rnd.random() < p_field * 0.8:
            r["dport"] = rnd.choice(port_pool)
        if rnd.random() < p_field * 0.3:
            k = rnd.sample(range(8), rnd.randint(1, 3))
            toks = [("!" if rnd.random() < 0.4 else "") + FLAGS[b] for b in k]
            if rnd.random() < 0.05:
                toks = []
            r["tcpflags"] = " ".join(toks)
        if ifaces and rnd.random() < p_field * 0.3:
            r["in_iface"] = rnd.choice(list(PORTS))
        if ifaces and rnd.random() < p_field * 0.3:
            r["out_iface"] = rnd.choice(list(PORTS))
        if ct and rnd.random() < p_field * 0.2:
            r["conntrack"] = rnd.choice(["NEW", "ESTABLISHED", "RELATED", "INVALID"])
        a = rnd.random()
        if a < 0.45:
            r["action"] = "DROP"
        elif a < 0.9:
            r["action"] = "ACCEPT"
        rules.append(r)
    return rules
