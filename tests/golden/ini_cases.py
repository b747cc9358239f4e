"""Rule files for the INI loader parity tests (reference src/rule_config.c:129-282): the
reference's own rules.example and test_suite.c:597-611 file, plus every accept / reject branch
and quirk of the loader.  (name, text, capacity)."""

SUITE = ("[rule]\npriority = 10\nprotocol = tcp\ndst_port = 80\naction = drop\n\n"
         "[rule]\npriority = 100\nip_version = 6\nsrc = 2001:db8::/32\naction = drop\n\n"
         "[rule]\npriority = 50000\naction = drop")


def cases(rules_example: str):
    r = "[rule]\n"
    return [
        ("rules_example", rules_example, 1024),
        ("test_suite", SUITE, 64),
        ("empty", "", 16),
        ("comments_ws", "# c\n; c\n\n   [rule]   \n  priority   =   7  \n action=drop\r\n", 16),
        ("rules_prefix_header", "[rules]\npriority = 3\naction = drop\n", 16),
        ("bad_header", "[rul]\npriority = 3\n", 16),
        ("outside_section", "priority = 3\n", 16),
        ("no_equals", r + "priority 3\n", 16),
        ("unknown_key", r + "colour = red\n", 16),
        ("bad_priority", r + "priority = -1\n", 16),
        ("bad_priority_text", r + "priority = 1x\n", 16),
        ("big_priority", r + "priority = 4294967297\naction = drop\n", 16),
        ("protocols", r + "protocol = icmpv6\n" + r + "protocol = 47\n" + r + "protocol = 300\n"
         + r + "protocol = abc\n" + r + "protocol = udp\n" + r + "protocol = icmp\n", 16),
        ("ip_version_bad", r + "ip_version = 5\n", 16),
        ("v4_host_and_prefix", r + "src = 10.1.2.3\ndst = 192.168.0.0/16\naction = drop\n", 16),
        ("v4_prefix_zero", r + "ip_version = 4\nsrc = 10.1.2.3/0\naction = drop\n", 16),
        ("prefix_wraps", r + "src = 10.0.0.0/288\naction = drop\n", 16),
        ("prefix_too_long", r + "src = 10.0.0.0/33\n", 16),
        ("prefix_negative", r + "src = 10.0.0.0/-1\n", 16),
        ("prefix_empty", r + "src = 10.0.0.0/\n", 16),
        ("v6_rules", r + "src = 2001:db8::1\ndst = fe80::/10\naction = drop\n"
         + r + "dst = ::/0\naction = drop\n", 16),
        ("mixed_version", r + "ip_version = 4\nsrc = 2001:db8::/32\naction = drop\n", 16),
        ("bad_address", r + "src = 10.0.0.256\n", 16),
        ("ports", r + "src_port = 0\ndst_port = 65535\naction = drop\n", 16),
        ("port_too_big", r + "dst_port = 65536\n", 16),
        ("fwd_no_iface", r + "action = fwd\n", 16),
        ("fwd_lo", r + "action = fwd\nout_iface = lo\n", 16),
        ("fwd_bad_iface", r + "action = fwd\nout_iface = nosuchif0\n", 16),
        ("bad_action", r + "action = accept\n", 16),
        ("override_keys", r + "priority = 5\npriority = 9\ndst_port = 1\ndst_port = 2\n"
         "action = drop\n", 16),
        ("same_priority_order", r + "priority = 5\ndst_port = 1\n" + r + "priority = 5\n"
         "dst_port = 2\n" + r + "priority = 1\ndst_port = 3\n", 16),
        ("capacity_overflow", (r + "priority = 1\n") * 3, 2),
        ("long_line", r + "priority = 1\n" + "# " + "x" * 700 + "\n" + "action = drop\n", 16),
    ]
