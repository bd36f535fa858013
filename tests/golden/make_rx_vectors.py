"""Writes tests/golden/rx_vectors.json: the known answers the reference itself states for the
receive-side filter. util/IPFilter.java:79-93 (IPFilter.main) builds a filter from
192.168.1.0/24 and 2001:db8::/32 and prints four searches with their expected results in
comments ("should return true/false"); allowingAll() (:67-77) inserts 0.0.0.0/32 and ::/128.
The expectations are transcribed here as data (the reference cannot be run: no JDK in the
image)."""
import json
import os

vectors = {
    "source": "util/IPFilter.java:79-93 (IPFilter.main expected outputs), :67-77 (allowingAll)",
    "filter": [["192.168.1.0", 24], ["2001:db8::", 32]],
    "search": [["192.168.1.55", True], ["192.168.2.1", False], ["2001:db8::abcd", True], ["2001:db9::abcd", False]],
    "allowing_all": [["0.0.0.0", 32], ["::", 128]],
}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "rx_vectors.json"), "w") as f:
    json.dump(vectors, f, indent=1)
