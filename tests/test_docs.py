"""The design documents cite measurements and code by path: every cited repo path must exist (a
renamed profile or moved tool would otherwise leave a dangling citation)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ['DESIGN.md', 'HISTORY.md', 'README.md', 'INTEGRATION.md', os.path.join('tools', 'README.md')]
CITED = re.compile(r'`((?:profiles|tools|tests|oracle|include|spatial-intention-maps_amd)/[^`\s]*)`')


@pytest.mark.parametrize('doc', DOCS)
def test_cited_paths_exist(doc):
    text = open(os.path.join(ROOT, doc)).read()
    missing = []
    for m in CITED.finditer(text):
        path = m.group(1).rstrip('.,;:)').split('::')[0]
        if '*' in path or '<' in path or path.startswith('oracle/_ref'):  # (built from /root/reference where it is mounted)
            continue
        if not os.path.exists(os.path.join(ROOT, path)):
            missing.append(path)
    assert not missing, missing
