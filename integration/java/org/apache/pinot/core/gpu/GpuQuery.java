package org.apache.pinot.core.gpu;

import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import org.apache.pinot.common.request.context.ExpressionContext;
import org.apache.pinot.common.request.context.FilterContext;
import org.apache.pinot.common.request.context.FunctionContext;
import org.apache.pinot.common.request.context.OrderByExpressionContext;
import org.apache.pinot.common.request.context.predicate.EqPredicate;
import org.apache.pinot.common.request.context.predicate.InPredicate;
import org.apache.pinot.common.request.context.predicate.NotEqPredicate;
import org.apache.pinot.common.request.context.predicate.NotInPredicate;
import org.apache.pinot.common.request.context.predicate.Predicate;
import org.apache.pinot.common.request.context.predicate.RangePredicate;
import org.apache.pinot.core.query.aggregation.function.AggregationFunction;
import org.apache.pinot.core.query.aggregation.function.DistinctCountHLLAggregationFunction;
import org.apache.pinot.core.query.request.context.QueryContext;
import org.apache.pinot.core.query.request.context.utils.QueryContextUtils;
import org.apache.pinot.segment.spi.AggregationFunctionType;


/**
 * QueryContext -> the ph_query descriptor of PinotHipJni.queryExecute (the Java twin of pinot_amd/query.py +
 * engine._QueryStruct).  Returns null for shapes outside the GPU path, so the plan maker keeps the CPU plan:
 * filtered aggregations, star-tree, null handling, non-identifier group-by expressions, aggregations other than
 * COUNT / SUM / MIN / MAX / DISTINCTCOUNTHLL (over a column or a 2-operand mult/sub/add), predicates other than
 * EQ / NOT_EQ / IN / NOT_IN / RANGE on identifiers, and a segment group trim (GroupByOperator.java:114-130) ordered
 * by anything but group-by columns and aggregations.
 */
public final class GpuQuery {
  final int[] _descriptor;
  final String[] _strings;
  final long _numGroupsLimit;
  final long _endTimeMs;

  private GpuQuery(int[] descriptor, String[] strings, long numGroupsLimit, long endTimeMs) {
    _descriptor = descriptor;
    _strings = strings;
    _numGroupsLimit = numGroupsLimit;
    _endTimeMs = endTimeMs;
  }

  public static GpuQuery compile(QueryContext ctx) {
    if (!QueryContextUtils.isAggregationQuery(ctx) || ctx.isNullHandlingEnabled() || ctx.hasFilteredAggregations()) {
      return null;
    }
    Builder b = new Builder();
    try {
      int root = ctx.getFilter() == null ? -1 : b.filter(ctx.getFilter());
      List<String> groupBy = new ArrayList<>();
      if (ctx.getGroupByExpressions() != null) {
        for (ExpressionContext e : ctx.getGroupByExpressions()) {
          if (e.getType() != ExpressionContext.Type.IDENTIFIER) {
            return null;
          }
          groupBy.add(e.getIdentifier());
        }
      }
      List<int[]> aggs = new ArrayList<>();
      for (AggregationFunction f : ctx.getAggregationFunctions()) {
        int[] a = b.aggregation(f);
        if (a == null) {
          return null;
        }
        aggs.add(a);
      }
      // [numFilterNodes, filterRoot, numPredicates, numGroupBy, numAggregations, nodes..., predicates...,
      //  group-by..., aggregations...]
      List<Integer> d = new ArrayList<>();
      d.add(b._nodes.size());
      d.add(root);
      d.add(b._preds.size());
      d.add(groupBy.size());
      d.add(aggs.size());
      for (int[] n : b._nodes) {
        for (int x : n) {
          d.add(x);
        }
      }
      for (int[] p : b._preds) {
        for (int x : p) {
          d.add(x);
        }
      }
      for (String g : groupBy) {
        d.add(b.str(g));
      }
      for (int[] a : aggs) {
        for (int x : a) {
          d.add(x);
        }
      }
      // [numOrderBy, (kind, index, asc)..., limit, minSegmentGroupTrimSize, skipStarTree]: segment group trim
      // (GroupByOperator.java:114-130) runs in the library (ph_query.min_segment_group_trim_size); a segment's
      // star-tree is taken there unless the skipStarTree query option is set (ph_query.skip_star_tree)
      List<OrderByExpressionContext> orderBy = ctx.getOrderByExpressions();
      List<int[]> order = new ArrayList<>();
      if (orderBy != null && ctx.getGroupByExpressions() != null) {
        for (OrderByExpressionContext ob : orderBy) {
          ExpressionContext e = ob.getExpression();
          int gi = ctx.getGroupByExpressions().indexOf(e);
          Integer ai = e.getType() == ExpressionContext.Type.FUNCTION
              ? ctx.getAggregationFunctionIndexMap().get(e.getFunction()) : null;
          if (gi >= 0) {
            order.add(new int[]{0, gi, ob.isAsc() ? 1 : 0});
          } else if (ai != null) {
            order.add(new int[]{1, ai, ob.isAsc() ? 1 : 0});
          } else if (ctx.getMinSegmentGroupTrimSize() > 0) {
            return null;  // an ORDER BY the trim cannot evaluate (expression over aggregations): CPU plan
          }
        }
      }
      d.add(order.size());
      for (int[] o : order) {
        for (int x : o) {
          d.add(x);
        }
      }
      d.add(ctx.getLimit());
      d.add(ctx.getMinSegmentGroupTrimSize());
      d.add(ctx.isSkipStarTree() ? 1 : 0);
      int[] desc = d.stream().mapToInt(Integer::intValue).toArray();
      return new GpuQuery(desc, b._strings.toArray(new String[0]), ctx.getNumGroupsLimit(), ctx.getEndTimeMs());
    } catch (UnsupportedOperationException e) {
      return null;
    }
  }

  /**
   * The descriptor of a WHERE clause alone, for ph_filter_execute (GpuFilterOperator): [numFilterNodes, filterRoot,
   * numPredicates, 0, 0, nodes..., predicates...]; null when a predicate is outside the GPU path.
   */
  public static GpuQuery compileFilter(FilterContext filter, long endTimeMs) {
    Builder b = new Builder();
    try {
      int root = b.filter(filter);
      List<Integer> d = new ArrayList<>();
      d.add(b._nodes.size());
      d.add(root);
      d.add(b._preds.size());
      d.add(0);
      d.add(0);
      for (int[] n : b._nodes) {
        for (int x : n) {
          d.add(x);
        }
      }
      for (int[] p : b._preds) {
        for (int x : p) {
          d.add(x);
        }
      }
      return new GpuQuery(d.stream().mapToInt(Integer::intValue).toArray(), b._strings.toArray(new String[0]), 0,
          endTimeMs);
    } catch (UnsupportedOperationException e) {
      return null;
    }
  }

  private static final class Builder {
    final List<int[]> _nodes = new ArrayList<>();
    final List<int[]> _preds = new ArrayList<>();
    final List<String> _strings = new ArrayList<>();
    final Map<String, Integer> _index = new HashMap<>();

    int str(String s) {
      return s == null ? -1 : _index.computeIfAbsent(s, k -> {
        _strings.add(k);
        return _strings.size() - 1;
      });
    }

    // FilterContext {AND, OR, NOT, PREDICATE} (FilterContext.java) -> ph_filter_node list, children first
    int filter(FilterContext f) {
      switch (f.getType()) {
        case AND:
        case OR:
        case NOT: {
          List<Integer> kids = new ArrayList<>();
          for (FilterContext c : f.getChildren()) {
            kids.add(filter(c));
          }
          int type = f.getType() == FilterContext.Type.AND ? PinotHipJni.FILTER_AND
              : f.getType() == FilterContext.Type.OR ? PinotHipJni.FILTER_OR : PinotHipJni.FILTER_NOT;
          int[] n = new int[3 + kids.size()];
          n[0] = type;
          n[1] = kids.size();
          n[2] = -1;
          for (int i = 0; i < kids.size(); i++) {
            n[3 + i] = kids.get(i);
          }
          _nodes.add(n);
          return _nodes.size() - 1;
        }
        case PREDICATE: {
          _nodes.add(new int[]{PinotHipJni.FILTER_PREDICATE, 0, predicate(f.getPredicate())});
          return _nodes.size() - 1;
        }
        default:
          throw new UnsupportedOperationException(f.getType().toString());
      }
    }

    // Predicate (pinot-common request/context/predicate) -> ph_predicate: values stay strings, as Pinot keeps them
    int predicate(Predicate p) {
      ExpressionContext lhs = p.getLhs();
      if (lhs.getType() != ExpressionContext.Type.IDENTIFIER) {
        throw new UnsupportedOperationException("predicate on an expression");
      }
      List<String> values = new ArrayList<>();
      int type;
      String lower = null;
      String upper = null;
      int lowerInc = 0;
      int upperInc = 0;
      switch (p.getType()) {
        case EQ:
          type = PinotHipJni.PRED_EQ;
          values.add(((EqPredicate) p).getValue());
          break;
        case NOT_EQ:
          type = PinotHipJni.PRED_NOT_EQ;
          values.add(((NotEqPredicate) p).getValue());
          break;
        case IN:
          type = PinotHipJni.PRED_IN;
          values.addAll(((InPredicate) p).getValues());
          break;
        case NOT_IN:
          type = PinotHipJni.PRED_NOT_IN;
          values.addAll(((NotInPredicate) p).getValues());
          break;
        case RANGE: {
          RangePredicate r = (RangePredicate) p;
          type = PinotHipJni.PRED_RANGE;
          lower = r.getLowerBound();   // RangePredicate.UNBOUNDED ("*") stays as is
          upper = r.getUpperBound();
          lowerInc = r.isLowerInclusive() ? 1 : 0;
          upperInc = r.isUpperInclusive() ? 1 : 0;
          break;
        }
        default:
          throw new UnsupportedOperationException(p.getType().toString());
      }
      int[] d = new int[7 + values.size()];
      int k = 0;
      d[k++] = type;
      d[k++] = str(lhs.getIdentifier());
      d[k++] = values.size();
      for (String v : values) {
        d[k++] = str(v);
      }
      d[k++] = str(lower);
      d[k++] = str(upper);
      d[k++] = lowerInc;
      d[k] = upperInc;
      _preds.add(d);
      return _preds.size() - 1;
    }

    // AggregationFunction -> {type, column, log2m, column2, exprOp} or null (not on the GPU path)
    int[] aggregation(AggregationFunction f) {
      AggregationFunctionType t = f.getType();
      List<ExpressionContext> in = f.getInputExpressions();
      if (t == AggregationFunctionType.COUNT) {
        return new int[]{PinotHipJni.AGG_COUNT, -1, 0, -1, PinotHipJni.EXPR_NONE};
      }
      int type;
      switch (t) {
        case SUM:
          type = PinotHipJni.AGG_SUM;
          break;
        case MIN:
          type = PinotHipJni.AGG_MIN;
          break;
        case MAX:
          type = PinotHipJni.AGG_MAX;
          break;
        case DISTINCTCOUNTHLL:
          type = PinotHipJni.AGG_DISTINCTCOUNTHLL;
          break;
        default:
          return null;
      }
      ExpressionContext e = in.get(0);
      int log2m = t == AggregationFunctionType.DISTINCTCOUNTHLL ? ((DistinctCountHLLAggregationFunction) f).getLog2m() : 0;
      if (e.getType() == ExpressionContext.Type.IDENTIFIER) {
        return new int[]{type, str(e.getIdentifier()), log2m, -1, PinotHipJni.EXPR_NONE};
      }
      // SUM(a*b) / SUM(a-b) / SUM(a+b): one 2-operand transform over identifiers (ProjectPlanNode.java:82)
      if (e.getType() == ExpressionContext.Type.FUNCTION && type != PinotHipJni.AGG_DISTINCTCOUNTHLL) {
        FunctionContext fn = e.getFunction();
        int op = "times".equals(fn.getFunctionName()) || "mult".equals(fn.getFunctionName()) ? PinotHipJni.EXPR_MULT
            : "minus".equals(fn.getFunctionName()) || "sub".equals(fn.getFunctionName()) ? PinotHipJni.EXPR_SUB
            : "plus".equals(fn.getFunctionName()) || "add".equals(fn.getFunctionName()) ? PinotHipJni.EXPR_ADD : -1;
        List<ExpressionContext> args = fn.getArguments();
        if (op > 0 && args.size() == 2 && args.get(0).getType() == ExpressionContext.Type.IDENTIFIER
            && args.get(1).getType() == ExpressionContext.Type.IDENTIFIER) {
          return new int[]{type, str(args.get(0).getIdentifier()), 0, str(args.get(1).getIdentifier()), op};
        }
      }
      return null;
    }
  }
}
