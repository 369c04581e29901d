"""Dictionary-based predicate evaluators (host side, per segment).

Restates the reference's evaluators, which run on the host before any scan:
  EQ      EqualsPredicateEvaluatorFactory.DictionaryBasedEqPredicateEvaluator (:92-123)
  NOT_EQ  NotEqualsPredicateEvaluatorFactory.DictionaryBasedNeqPredicateEvaluator
  IN      InPredicateEvaluatorFactory.DictionaryBasedInPredicateEvaluator (:158-200),
          PredicateUtils.getDictIdSet (:78-92)
  NOT_IN  NotInPredicateEvaluatorFactory.DictionaryBasedNotInPredicateEvaluator
  RANGE   RangePredicateEvaluatorFactory.SortedDictionaryBasedRangePredicateEvaluator (:119-246)
(all under pinot-core/src/main/java/org/apache/pinot/core/operator/filter/predicate/).

The outcome is what the GPU plan carries per segment: always-true / always-false, a dict-id
range [start, end), or a dict-id set (exclusive = the predicate matches the complement).
"""
from dataclasses import dataclass
from typing import Tuple

from ..segment.dictionary import Dictionary
from .context import Predicate, PredicateType, UNBOUNDED


@dataclass
class DictPredicateEvaluation:
    always_true: bool = False
    always_false: bool = False
    kind: str = "range"            # "range" | "set"
    start: int = 0                 # range: [start, end)
    end: int = 0
    ids: Tuple[int, ...] = ()      # set: dict ids (sorted)
    exclusive: bool = False        # set: match dict ids NOT in ids

    def matching_dict_ids(self, cardinality):
        if self.always_false:
            return []
        if self.always_true:
            return list(range(cardinality))
        if self.kind == "range":
            return list(range(self.start, self.end))
        if self.exclusive:
            s = set(self.ids)
            return [i for i in range(cardinality) if i not in s]
        return list(self.ids)


def _ids_of(dictionary: Dictionary, values):
    ids = set()
    for v in values:
        i = dictionary.index_of(v)
        if i >= 0:
            ids.add(i)
    return tuple(sorted(ids))


def evaluate(pred: Predicate, dictionary: Dictionary) -> DictPredicateEvaluation:
    card = len(dictionary)
    t = pred.type
    if t == PredicateType.EQ:
        i = dictionary.index_of(pred.values[0])
        if i < 0:
            return DictPredicateEvaluation(always_false=True)
        return DictPredicateEvaluation(always_true=(card == 1), kind="range", start=i, end=i + 1)
    if t == PredicateType.NOT_EQ:
        i = dictionary.index_of(pred.values[0])
        if i < 0:
            return DictPredicateEvaluation(always_true=True)
        if card == 1:
            return DictPredicateEvaluation(always_false=True)
        return DictPredicateEvaluation(kind="set", ids=(i,), exclusive=True)
    if t == PredicateType.IN:
        ids = _ids_of(dictionary, pred.values)
        if not ids:
            return DictPredicateEvaluation(always_false=True)
        if len(ids) == card:
            return DictPredicateEvaluation(always_true=True)
        if ids[-1] - ids[0] + 1 == len(ids):
            return DictPredicateEvaluation(kind="range", start=ids[0], end=ids[-1] + 1)
        return DictPredicateEvaluation(kind="set", ids=ids)
    if t == PredicateType.NOT_IN:
        ids = _ids_of(dictionary, pred.values)
        if not ids:
            return DictPredicateEvaluation(always_true=True)
        if len(ids) == card:
            return DictPredicateEvaluation(always_false=True)
        return DictPredicateEvaluation(kind="set", ids=ids, exclusive=True)
    if t == PredicateType.RANGE:
        # SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:126-169)
        if pred.lower == UNBOUNDED:
            start = 0
        else:
            ii = dictionary.insertion_index_of(pred.lower)
            if ii < 0:
                start = -(ii + 1)
            else:
                start = ii if pred.lower_inclusive else ii + 1
        if pred.upper == UNBOUNDED:
            end = card
        else:
            ii = dictionary.insertion_index_of(pred.upper)
            if ii < 0:
                end = -(ii + 1)
            else:
                end = ii + 1 if pred.upper_inclusive else ii
        n = max(end - start, 0)
        if n == 0:
            return DictPredicateEvaluation(always_false=True)
        if n == card:
            return DictPredicateEvaluation(always_true=True)
        return DictPredicateEvaluation(kind="range", start=start, end=end)
    raise NotImplementedError(t)
