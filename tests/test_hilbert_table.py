"""The query order's Hilbert state table (sort.hip kHilbertTable) is the Skilling transform it replaces
(scripts/sort_debug.py hilbert24, the numpy copy of the transform the query-order GPU test checks against)."""
from scripts import hilbert_table as H


def test_table_in_source_is_the_derived_one():
    assert H.table_in_source() == H.derive()


def test_table_equals_transform_on_every_cell():
    assert H.check(H.table_in_source())
