"""CPU: pin the oracle restatement against the reference-generated goldens."""
import numpy as np
import pytest

import oracle
from goldens import CASE_NAMES, check_dups, check_perm, load_case


@pytest.fixture(scope="module", params=CASE_NAMES)
def case(request, built):
    return load_case(request.param)


def test_oracle_sort_matches_reference(case):
    perm = oracle.sort_perm(case.recs, case.offs, case.n)
    check_perm(case, perm)


def test_oracle_dedup_sorted_verbose(case):
    perm = oracle.sort_perm(case.recs, case.offs, case.n)
    dup, nd = oracle.markdup(case.recs, case.offs[:-1][perm], case.n, case.header)
    check_dups(case, "dedup_sorted_v", dup, case.offs[:-1][perm])


def test_oracle_dedup_input_verbose(case):
    dup, nd = oracle.markdup(case.recs, case.offs, case.n, case.header)
    check_dups(case, "dedup_input_v", dup, case.offs)


def test_oracle_dedup_input_nonverbose_quirk(case):
    """without -v the record index never advances, so at most record 0 is flagged."""
    dup, nd = oracle.markdup(case.recs, case.offs, case.n, case.header, compat_nonverbose=True)
    check_dups(case, "dedup_input_nv", dup, case.offs)
    assert nd <= 1


@pytest.mark.parametrize("k", [3, 12])
def test_oracle_dedup_split_chains(case, k):
    """the reference's default split-by-chromosome chains (dedup without --nosplit)."""
    perm = oracle.sort_perm(case.recs, case.offs, case.n)
    dup, nd = oracle.markdup(case.recs, case.offs[:-1][perm], case.n, case.header, split_chains=k)
    check_dups(case, f"dedup_sorted_v_k{k}", dup, case.offs[:-1][perm])


def test_yhet208_survey_count():
    """The survey's independent run of the reference: 6,642 duplicates on sorted 208.yhet.bam with -v."""
    case = load_case("yhet208")
    perm = oracle.sort_perm(case.recs, case.offs, case.n)
    dup, nd = oracle.markdup(case.recs, case.offs[:-1][perm], case.n, case.header)
    assert nd == 6642
