"""The online-boutique workload: every message of the reference's
benchmark/serialization/online-boutique/proto/onlineboutique.proto as a run-time schema of
arpc_amd.flat, and the JSON payloads the reference benchmark loads turned into device columns.

Reference: onlineboutique.proto (33 messages; no field sets is_public, so every field is private)
and its generated codec onlineboutique.syn.go (e.g. CartItem :83-144, Cart :1361-1457, Empty
:1742-1751).  The benchmark (bench_test.go:282-351) marshals / unmarshals the payloads one message
per call after loader.go parsed each JSONL line with protojson (DiscardUnknown): fields are named by
their proto names (snake_case), int64 may be a JSON string, an absent field is the zero value, a
present message (even `{}`) is non-nil.  Here a batch is all the messages of one type.

Schemas list the fields in declaration order with their Go names (the generator's order,
main.go:1172-1210); `json` maps a Go name to its proto name.
"""
from __future__ import annotations

import numpy as np

from .flat import FlatField as F, FlatSchema as S, columns_from_tree

# ---- onlineboutique.proto, in file order -------------------------------------------------------
CART_ITEM = S("CartItem", (F("ProductId", "string"), F("Quantity", "int32")))
ADD_ITEM_REQUEST = S("AddItemRequest", (F("UserId", "string"), F("Item", "message", message=CART_ITEM)))
EMPTY_CART_REQUEST = S("EmptyCartRequest", (F("UserId", "string"),))
GET_CART_REQUEST = S("GetCartRequest", (F("UserId", "string"),))
CART = S("Cart", (F("UserId", "string"), F("Items", "message", repeated=True, message=CART_ITEM)))
EMPTY = S("Empty", ())
EMPTY_USER = S("EmptyUser", (F("UserId", "string"),))
LIST_RECOMMENDATIONS_REQUEST = S("ListRecommendationsRequest", (F("UserId", "string"),
                                                                 F("ProductIds", "string", repeated=True)))
LIST_RECOMMENDATIONS_RESPONSE = S("ListRecommendationsResponse", (F("ProductIds", "string", repeated=True),))
MONEY = S("Money", (F("CurrencyCode", "string"), F("Units", "int64"), F("Nanos", "int32")))
PRODUCT = S("Product", (F("Id", "string"), F("Name", "string"), F("Description", "string"), F("Picture", "string"),
                        F("PriceUsd", "message", message=MONEY), F("Categories", "string", repeated=True)))
LIST_PRODUCTS_RESPONSE = S("ListProductsResponse", (F("Products", "message", repeated=True, message=PRODUCT),))
GET_PRODUCT_REQUEST = S("GetProductRequest", (F("Id", "string"),))
SEARCH_PRODUCTS_REQUEST = S("SearchProductsRequest", (F("Query", "string"),))
SEARCH_PRODUCTS_RESPONSE = S("SearchProductsResponse", (F("Results", "message", repeated=True, message=PRODUCT),))
ADDRESS = S("Address", (F("StreetAddress", "string"), F("City", "string"), F("State", "string"),
                        F("Country", "string"), F("ZipCode", "int32")))
GET_QUOTE_REQUEST = S("GetQuoteRequest", (F("Address", "message", message=ADDRESS),
                                          F("Items", "message", repeated=True, message=CART_ITEM)))
GET_QUOTE_RESPONSE = S("GetQuoteResponse", (F("CostUsd", "message", message=MONEY),))
SHIP_ORDER_REQUEST = S("ShipOrderRequest", (F("Address", "message", message=ADDRESS),
                                            F("Items", "message", repeated=True, message=CART_ITEM)))
SHIP_ORDER_RESPONSE = S("ShipOrderResponse", (F("TrackingId", "string"),))
GET_SUPPORTED_CURRENCIES_RESPONSE = S("GetSupportedCurrenciesResponse", (F("CurrencyCodes", "string", repeated=True),))
CURRENCY_CONVERSION_REQUEST = S("CurrencyConversionRequest", (F("From", "message", message=MONEY),
                                                              F("ToCode", "string"), F("UserId", "string")))
CREDIT_CARD_INFO = S("CreditCardInfo", (F("CreditCardNumber", "string"), F("CreditCardCvv", "int32"),
                                        F("CreditCardExpirationYear", "int32"), F("CreditCardExpirationMonth", "int32")))
CHARGE_REQUEST = S("ChargeRequest", (F("Amount", "message", message=MONEY),
                                     F("CreditCard", "message", message=CREDIT_CARD_INFO)))
CHARGE_RESPONSE = S("ChargeResponse", (F("TransactionId", "string"),))
ORDER_ITEM = S("OrderItem", (F("Item", "message", message=CART_ITEM), F("Cost", "message", message=MONEY)))
ORDER_RESULT = S("OrderResult", (F("OrderId", "string"), F("ShippingTrackingId", "string"),
                                 F("ShippingCost", "message", message=MONEY),
                                 F("ShippingAddress", "message", message=ADDRESS),
                                 F("Items", "message", repeated=True, message=ORDER_ITEM)))
SEND_ORDER_CONFIRMATION_REQUEST = S("SendOrderConfirmationRequest", (F("Email", "string"),
                                                                     F("Order", "message", message=ORDER_RESULT)))
PLACE_ORDER_REQUEST = S("PlaceOrderRequest", (F("UserId", "string"), F("UserCurrency", "string"),
                                              F("Address", "message", message=ADDRESS), F("Email", "string"),
                                              F("CreditCard", "message", message=CREDIT_CARD_INFO)))
PLACE_ORDER_RESPONSE = S("PlaceOrderResponse", (F("Order", "message", message=ORDER_RESULT),))
AD_REQUEST = S("AdRequest", (F("UserId", "string"), F("ContextKeys", "string", repeated=True)))
AD = S("Ad", (F("RedirectUrl", "string"), F("Text", "string")))
AD_RESPONSE = S("AdResponse", (F("Ads", "message", repeated=True, message=AD),))

SCHEMAS = {s.name: s for s in (
    CART_ITEM, ADD_ITEM_REQUEST, EMPTY_CART_REQUEST, GET_CART_REQUEST, CART, EMPTY, EMPTY_USER,
    LIST_RECOMMENDATIONS_REQUEST, LIST_RECOMMENDATIONS_RESPONSE, PRODUCT, LIST_PRODUCTS_RESPONSE, GET_PRODUCT_REQUEST,
    SEARCH_PRODUCTS_REQUEST, SEARCH_PRODUCTS_RESPONSE, GET_QUOTE_REQUEST, GET_QUOTE_RESPONSE, SHIP_ORDER_REQUEST,
    SHIP_ORDER_RESPONSE, ADDRESS, MONEY, GET_SUPPORTED_CURRENCIES_RESPONSE, CURRENCY_CONVERSION_REQUEST,
    CREDIT_CARD_INFO, CHARGE_REQUEST, CHARGE_RESPONSE, ORDER_ITEM, ORDER_RESULT, SEND_ORDER_CONFIRMATION_REQUEST,
    PLACE_ORDER_REQUEST, PLACE_ORDER_RESPONSE, AD_REQUEST, AD, AD_RESPONSE)}


def json_name(go: str) -> str:
    """protoc-gen-go's CamelCase name back to the proto field name (ProductId -> product_id)."""
    out = []
    for k, c in enumerate(go):
        if c.isupper() and k:
            out.append("_")
        out.append(c.lower())
    return "".join(out)


_NP = {"bool": np.uint8, "int32": np.int32, "uint32": np.uint32, "float": np.float32, "enum": np.int32,
       "int64": np.int64, "uint64": np.uint64, "double": np.float64}


def _scalar(kind: str, v):
    """A JSON value of a protobuf scalar as protojson reads it (64-bit integers may be strings)."""
    if v is None:
        return 0
    if kind == "bool":
        return 1 if v else 0
    if kind in ("float", "double"):
        return float(v)
    return int(v)


def _packed(vals: list):
    off = np.zeros(len(vals) + 1, np.int64)
    np.cumsum([len(v) for v in vals], out=off[1:])
    return np.frombuffer(b"".join(vals), np.uint8).copy(), off


def tree_from_json(schema: S, msgs: list) -> list:
    """JSON objects of one message type -> the host column tree of arpc_amd.flat.columns_from_tree
    (one node per field, recursively)."""
    nodes = []
    for f in schema.fields:
        key = json_name(f.name)
        vals = [m.get(key) for m in msgs]
        if f.kind == "message":
            items, counts = [], []
            for v in vals:
                its = (v or []) if f.repeated else ([] if v is None else [v])
                items.extend(its)
                counts.append(len(its))
            rec = np.zeros(len(msgs) + 1, np.int64)
            np.cumsum(counts, out=rec[1:])
            nodes.append(("msg", tree_from_json(f.message, items), rec))
        elif f.repeated and f.kind in ("string", "bytes"):
            items = [s.encode() if isinstance(s, str) else bytes(s) for v in vals for s in (v or [])]
            rec = np.zeros(len(msgs) + 1, np.int64)
            np.cumsum([len(v or []) for v in vals], out=rec[1:])
            b, io = _packed(items)
            nodes.append(("list", b, io, rec))
        elif f.repeated:  # repeated scalar: the elements' bytes per record
            b, o = _packed([np.array([_scalar(f.kind, x) for x in (v or [])], _NP[f.kind]).tobytes() for v in vals])
            nodes.append((b, o))
        elif f.kind in ("string", "bytes"):
            nodes.append(_packed([(v or "").encode() if not isinstance(v, bytes) else v for v in vals]))
        else:
            nodes.append(np.array([_scalar(f.kind, v) for v in vals], _NP[f.kind]))
    return nodes


def columns_from_json(schema: S, msgs: list, device) -> list:
    """JSON objects of one message type -> device columns for arpc_amd.flat.encode."""
    return columns_from_tree(schema, tree_from_json(schema, msgs), device)
