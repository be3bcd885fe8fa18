"""TPC-H schema and the constant value lists of the TPC-H spec (§4.2.2-4.2.3).

Used by the synthetic generator (datagen.py). Storage types are chosen for
HBM bandwidth: keys are INT32 (every SF<=1000 key fits), money/quantities are
DECIMAL(15,2) as scaled int64, dates DATE32, and low-cardinality strings are
dictionary-encoded.
"""
from __future__ import annotations

NATIONS = [
    ("ALGERIA", 0), ("ARGENTINA", 1), ("BRAZIL", 1), ("CANADA", 1), ("EGYPT", 4), ("ETHIOPIA", 0), ("FRANCE", 3),
    ("GERMANY", 3), ("INDIA", 2), ("INDONESIA", 2), ("IRAN", 4), ("IRAQ", 4), ("JAPAN", 2), ("JORDAN", 4),
    ("KENYA", 0), ("MOROCCO", 0), ("MOZAMBIQUE", 0), ("PERU", 1), ("CHINA", 2), ("ROMANIA", 3),
    ("SAUDI ARABIA", 4), ("VIETNAM", 2), ("RUSSIA", 3), ("UNITED KINGDOM", 3), ("UNITED STATES", 1),
]
REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]

COLORS = ("almond antique aquamarine azure beige bisque black blanched blue blush brown burlywood burnished "
          "chartreuse chiffon chocolate coral cornflower cornsilk cream cyan dark deep dim dodger drab firebrick "
          "floral forest frosted gainsboro ghost goldenrod green grey honeydew hot indian ivory khaki lace lavender "
          "lawn lemon light lime linen magenta maroon medium metallic midnight mint misty moccasin navajo navy "
          "olive orange orchid pale papaya peach peru pink plum powder puff purple red rose rosy royal saddle "
          "salmon sandy seashell sienna sky slate smoke snow spring steel tan thistle tomato turquoise violet "
          "wheat white yellow").split()

TYPE_S1 = ["STANDARD", "SMALL", "MEDIUM", "LARGE", "ECONOMY", "PROMO"]
TYPE_S2 = ["ANODIZED", "BURNISHED", "PLATED", "POLISHED", "BRUSHED"]
TYPE_S3 = ["TIN", "NICKEL", "BRASS", "STEEL", "COPPER"]
CONT_S1 = ["SM", "LG", "MED", "JUMBO", "WRAP"]
CONT_S2 = ["CASE", "BOX", "BAG", "JAR", "PKG", "PACK", "CAN", "DRUM"]
SEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
PRIORITIES = ["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"]
INSTRUCTIONS = ["DELIVER IN PERSON", "COLLECT COD", "NONE", "TAKE BACK RETURN"]
MODES = ["REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"]

# comment vocabulary (TPC-H text grammar word classes)
WORDS = ("foxes ideas theodolites pinto beans instructions dependencies excuses platelets asymptotes courts "
         "dolphins multipliers sauternes warthogs frets dinos attainments somas Tiresias patterns forges braids "
         "hockey players frays warhorses dugouts notornis epitaphs pearls tithes waters orbits gifts sheaves "
         "depths sentiments decoys realms pains grouches escapades packages requests accounts deposits "
         "sleep wake are cajole haggle nag use boost affix detect integrate maintain nod was lose sublate solve "
         "thrash promise engage hinder print x-ray breach eat grow impress mold poach serve run dazzle snooze "
         "doze unwind kindle play hang believe doubt furious sly careful blithe quick fluffy slow quiet ruthless "
         "thin close dogged daring brave stealthy permanent enticing idle busy regular final ironic even bold "
         "silent special pending unusual express sometimes always never furiously slyly carefully blithely "
         "quickly fluffily slowly quietly ruthlessly thinly closely doggedly daringly bravely stealthily "
         "permanently enticingly idly busily regularly finally ironically evenly boldly silently about above "
         "according across after against along alongside among around at atop before behind beneath beside "
         "besides between beyond by despite during except for from inside instead into near of on outside over "
         "past since through throughout to toward under until up upon without with within the").split()

START_DATE = "1992-01-01"
END_DATE = "1998-12-31"
CURRENT_DATE = "1995-06-17"

TABLES = ["region", "nation", "supplier", "customer", "part", "partsupp", "orders", "lineitem"]

# primary keys (used by the planner's statistics and the distributed layout)
PRIMARY_KEYS = {
    "region": ["r_regionkey"], "nation": ["n_nationkey"], "supplier": ["s_suppkey"], "customer": ["c_custkey"],
    "part": ["p_partkey"], "partsupp": ["ps_partkey", "ps_suppkey"], "orders": ["o_orderkey"],
    "lineitem": ["l_orderkey", "l_linenumber"],
}
# hash-partitioning column of each table across ranks (None = replicated)
PARTITION_KEY = {
    "region": None, "nation": None, "supplier": "s_suppkey", "customer": "c_custkey", "part": "p_partkey",
    "partsupp": "ps_partkey", "orders": "o_orderkey", "lineitem": "l_orderkey",
}


def row_counts(sf: float) -> dict:
    return {
        "region": 5, "nation": 25, "supplier": int(10_000 * sf), "customer": int(150_000 * sf),
        "part": int(200_000 * sf), "partsupp": int(800_000 * sf), "orders": int(1_500_000 * sf),
        "lineitem": None,  # ~6M * sf, 1..7 per order
    }
