"""IANA code translation (oni-oa components/iana): DNS qtype / qclass /
rcode and HTTP status codes → names. Static tables (the reference shipped CSVs)."""
from __future__ import annotations

DNS_TYPES = {1: "A", 2: "NS", 5: "CNAME", 6: "SOA", 10: "NULL", 12: "PTR", 13: "HINFO", 15: "MX", 16: "TXT",
             17: "RP", 18: "AFSDB", 24: "SIG", 25: "KEY", 28: "AAAA", 29: "LOC", 33: "SRV", 35: "NAPTR", 36: "KX",
             37: "CERT", 39: "DNAME", 41: "OPT", 42: "APL", 43: "DS", 44: "SSHFP", 45: "IPSECKEY", 46: "RRSIG",
             47: "NSEC", 48: "DNSKEY", 49: "DHCID", 50: "NSEC3", 51: "NSEC3PARAM", 52: "TLSA", 55: "HIP",
             59: "CDS", 60: "CDNSKEY", 61: "OPENPGPKEY", 64: "SVCB", 65: "HTTPS", 99: "SPF", 249: "TKEY",
             250: "TSIG", 251: "IXFR", 252: "AXFR", 255: "ANY", 256: "URI", 257: "CAA", 32768: "TA", 32769: "DLV"}
DNS_CLASSES = {1: "IN", 3: "CH", 4: "HS", 254: "NONE", 255: "ANY"}
DNS_RCODES = {0: "NoError", 1: "FormErr", 2: "ServFail", 3: "NXDomain", 4: "NotImp", 5: "Refused", 6: "YXDomain",
              7: "YXRRSet", 8: "NXRRSet", 9: "NotAuth", 10: "NotZone", 16: "BADVERS", 17: "BADKEY", 18: "BADTIME",
              19: "BADMODE", 20: "BADNAME", 21: "BADALG", 22: "BADTRUNC", 23: "BADCOOKIE"}
HTTP_STATUS = {100: "Continue", 101: "Switching Protocols", 200: "OK", 201: "Created", 202: "Accepted",
               204: "No Content", 206: "Partial Content", 301: "Moved Permanently", 302: "Found",
               303: "See Other", 304: "Not Modified", 307: "Temporary Redirect", 308: "Permanent Redirect",
               400: "Bad Request", 401: "Unauthorized", 403: "Forbidden", 404: "Not Found",
               405: "Method Not Allowed", 407: "Proxy Authentication Required", 408: "Request Timeout",
               409: "Conflict", 410: "Gone", 413: "Payload Too Large", 414: "URI Too Long", 429: "Too Many Requests",
               500: "Internal Server Error", 501: "Not Implemented", 502: "Bad Gateway", 503: "Service Unavailable",
               504: "Gateway Timeout"}


def dns_type(v: int) -> str:
    return DNS_TYPES.get(int(v), str(v))


def dns_class(v: int) -> str:
    return DNS_CLASSES.get(int(v), str(v))


def dns_rcode(v: int) -> str:
    return DNS_RCODES.get(int(v), str(v))


def http_status(v: int) -> str:
    return HTTP_STATUS.get(int(v), str(v))
