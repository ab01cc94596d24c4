"""Column specs for raw telemetry tables, ML results CSVs and OA score/feedback CSVs.

Table-driven on purpose: the reference's exact CSV column orders are not verifiable from the
snapshot, so every order lives here and nowhere else.

Raw schemas ([U-M]):
* flow  -- nfdump CSV fields as loaded into the Hive ``flow`` table;
* dns   -- tshark DNS-response fields;
* proxy -- Bluecoat access-log fields.
"""
from __future__ import annotations

FLOW_COLUMNS = [
    "treceived", "unix_tstamp", "tryear", "trmonth", "trday", "trhour", "trminute", "trsec", "tdur",
    "sip", "dip", "sport", "dport", "proto", "flag", "fwd", "stos", "ipkt", "ibyt", "opkt", "obyt",
    "input", "output", "sas", "das", "dtos", "dir", "rip",
]
FLOW_IP_COLUMNS = {"sip", "dip", "rip"}
FLOW_FLOAT_COLUMNS = {"tdur"}
FLOW_TIME_COLUMNS = {"treceived"}  # rendered "YYYY-MM-DD HH:MM:SS"

DNS_COLUMNS = [
    "frame_time", "unix_tstamp", "frame_len", "ip_src", "ip_dst", "dns_qry_name", "dns_qry_type",
    "dns_qry_class", "dns_qry_rcode", "dns_a",
]

PROXY_COLUMNS = [
    "p_date", "p_time", "clientip", "host", "reqmethod", "useragent", "resconttype", "duration", "username",
    "authgroup", "exceptionid", "filterresult", "webcat", "referer", "respcode", "action", "urischeme",
    "uriport", "uripath", "uriquery", "uriextension", "serverip", "scbytes", "csbytes", "virusid",
    "bcappname", "bcappoperation", "fulluri",
]

# ML results (= raw columns in schema order + derived words + scores), ascending by score
FLOW_RESULT_COLUMNS = FLOW_COLUMNS + ["src_word", "dst_word", "src_score", "dst_score", "score"]
DNS_RESULT_COLUMNS = DNS_COLUMNS + ["word", "score"]
PROXY_RESULT_COLUMNS = PROXY_COLUMNS + ["word", "score"]

# OA scores / feedback files: first column is the analyst severity
# sev: 0 = unscored, 1 = high risk, 2 = medium, 3 = low risk (benign -> feedback "noise filter")
FLOW_SCORE_COLUMNS = [
    "sev", "tstart", "srcIP", "dstIP", "sport", "dport", "proto", "ipkt", "ibyt", "srcGeo", "dstGeo",
    "srcDomain", "dstDomain", "srcIP_rep", "dstIP_rep",
]
DNS_SCORE_COLUMNS = [
    "sev", "frame_time", "frame_len", "ip_dst", "dns_qry_name", "dns_qry_class", "dns_qry_type",
    "dns_qry_rcode", "domain", "subdomain", "subdomain_length", "num_periods", "subdomain_entropy",
    "top_domain", "word", "score", "query_rep", "hh", "ip_sev", "dns_sev", "dns_qry_class_name",
    "dns_qry_type_name", "dns_qry_rcode_name", "network_context", "unix_tstamp",
]
PROXY_SCORE_COLUMNS = [
    "sev", "p_date", "p_time", "clientip", "host", "reqmethod", "useragent", "resconttype", "duration",
    "username", "webcat", "referer", "respcode", "uriport", "uripath", "uriquery", "serverip", "scbytes",
    "csbytes", "fulluri", "word", "score", "uri_rep", "respcode_name", "network_context",
]

SEV_UNSCORED, SEV_HIGH, SEV_MEDIUM, SEV_LOW = 0, 1, 2, 3

SOURCES = ("flow", "dns", "proxy")


def result_columns(source: str) -> list[str]:
    return {"flow": FLOW_RESULT_COLUMNS, "dns": DNS_RESULT_COLUMNS, "proxy": PROXY_RESULT_COLUMNS}[source]


def raw_columns(source: str) -> list[str]:
    return {"flow": FLOW_COLUMNS, "dns": DNS_COLUMNS, "proxy": PROXY_COLUMNS}[source]


def score_columns(source: str) -> list[str]:
    return {"flow": FLOW_SCORE_COLUMNS, "dns": DNS_SCORE_COLUMNS, "proxy": PROXY_SCORE_COLUMNS}[source]
